#!/bin/bash
# One parameterised GPU-box driver (replaces the round-3 one-off gpu_cmd_*.sh scripts).
#   gpurun -- 'bash tools/gpu_steps.sh OUT step [step ...]'
# Steps (each under its own time limit; the first failure ends the run):
#   suite          pytest -m gpu (the whole GPU suite)
#   test=EXPR      pytest -m gpu -k EXPR
#   smoke          __graft_entry__.smoke()
#   bench          the default bench.py line (CPU baseline and secondaries included)
#   quick          bench.py --no-cpu --no-secondary --steps 3 --warmup 1
#   ab=V1,V2,...   tools/ab_quick.sh over library variants ("main" = herdsman_amd/lib)
#   abk=V1,V2,...  per-kernel A/B: rocprofv3 --kernel-trace --stats of op_bench ckks_mul per variant,
#                  2 reps interleaved, then tools/kstat_cmp.py (op rate in each variant's log)
#   stats          rocprofv3 --kernel-trace --stats of a short bench.py (roofline summary)
#   steppmc[=OP]   kernel trace + FETCH_SIZE + WRITE_SIZE passes of op_bench OP (default ckks_mul, 128 per call):
#                  summarise here with tools/step_summary.py -> profiles/<round>/step_summary.json
#   optrace=OP     rocprofv3 --kernel-trace --stats of tools/op_bench.py OP (bfv_mul, ckks_mul, ckks_rot)
#   prof           tools/profile_round.sh (roofline stats, PMC passes; summarise with tools/collect_profile.py)
#   steptable      rocprofv3 kernel trace of one C5 wave loop -> tools/step_table.py
#   valu=V1,V2     SQ_INSTS_VALU + SQ_WAVES of op_bench ckks_mul (128 per call) per variant -> tools/valu_count.py
#   valuop=OP:V1,V2  the same for another op_bench op (bfv_mul, ckks_rot, ...)
#   abop=OP:V1,V2  op_bench OP (128 per call, 20 reps) per variant, 3 interleaved reps ("OP+f": --openfhe-primes)
#   wgbench        GpuWorkerGroup MapTask throughput end to end (wg_run bench, files under /tmp on the box)
set -e
export TMPDIR=/tmp
O=$1; shift
mkdir -p "$O"
for s in "$@"; do
  echo "== $s $(date +%T)"
  case $s in
    suite) timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gputests.log" 2>&1 ;;
    test=*) timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${s#test=}" > "$O/gputest_${s#test=}.log" 2>&1 ;;
    smoke) timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 ;;
    bench) timeout -k 10 600 python3 bench.py > "$O/bench.log" 2>&1 ;;
    quick) timeout -k 10 300 python3 bench.py --no-cpu --no-secondary --steps 3 --warmup 1 > "$O/quick.log" 2>&1 ;;
    ab=*) IFS=, read -r -a vs <<< "${s#ab=}"; bash tools/ab_quick.sh "$O/q" "${vs[@]}" > "$O/ab.txt" 2>&1 ;;
    abk=*) IFS=, read -r -a vs <<< "${s#abk=}"
      lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
      for v in "${vs[@]}"; do  # parity first: the digests and the metric-config parity cases
        HERD_FHE_LIB=$(lib_of $v) timeout -k 10 300 python3 -u -m pytest tests/test_digests.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/parity.$v.log" 2>&1
        echo "$v parity: $(tail -n 1 "$O/parity.$v.log")"
      done
      for v in "${vs[@]}"; do
        HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/k/$v" -o run -- python3 tools/op_bench.py ckks_mul --batch 128 --reps 5 > "$O/k.$v.log" 2>&1
        f=$(find "$O/k/$v" -name run_kernel_stats.csv | head -n 1); cp "$f" "$O/k/$v/run_kernel_stats.csv" 2>/dev/null || true
      done
      python3 tools/kstat_cmp.py "$O/k" "${vs[@]}" > "$O/kcmp.txt"
      for rep in 1 2 3; do for v in "${vs[@]}"; do
        echo "$v rep$rep $(HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py ckks_mul --batch 128 --reps 20 2>/dev/null | tail -n 1)"
      done; done > "$O/abk.txt" ;;
    stats) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats" -o run -- python3 bench.py --no-cpu --no-secondary --steps 3 --warmup 1 > "$O/stats.log" 2>&1 ;;
    steppmc|steppmc=*)
      OPP=ckks_mul; [ "$s" = steppmc ] || OPP=${s#steppmc=}
      B="python3 tools/op_bench.py $OPP --batch 128"
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/st_trace" -o run -- $B --reps 4 > "$O/st_trace.log" 2>&1
      timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/st_fetch" -o run -- $B --reps 2 > "$O/st_fetch.log" 2>&1
      timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/st_write" -o run -- $B --reps 2 > "$O/st_write.log" 2>&1 ;;
    optrace=*) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/op_${s#optrace=}" -o run -- python3 tools/op_bench.py "${s#optrace=}" --batch 128 --reps 5 > "$O/op_${s#optrace=}.log" 2>&1 ;;
    prof) timeout -k 10 1100 bash tools/profile_round.sh "$O/prof" > "$O/prof.log" 2>&1 ;;
    wgbench) rm -rf /tmp/wgb && timeout -k 10 400 herdsman_amd/bin/wg_run bench /tmp/wgb 0,16,12,4,3,0 4 64 4 16 6 > "$O/wg_bench.log" 2>&1; rm -rf /tmp/wgb ;;
    valu=*|valuop=*)
      if [ "${s%%=*}" = valuop ]; then spec=${s#valuop=}; OP=${spec%%:*}; VS=${spec#*:}; else OP=ckks_mul; VS=${s#valu=}; fi
      IFS=, read -r -a vs <<< "$VS"
      lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
      for v in "${vs[@]}"; do
        HERD_FHE_LIB=$(lib_of $v) timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d "$O/valu_$OP/$v" -o run -- python3 tools/op_bench.py $OP --batch 128 --reps 2 > "$O/valu_$OP.$v.log" 2>&1
      done
      python3 tools/valu_count.py "$O/valu_$OP" "${vs[@]}" > "$O/valu_$OP.txt" 2>&1 || true ;;
    abop=*)
      spec=${s#abop=}; OP=${spec%%:*}; IFS=, read -r -a vs <<< "${spec#*:}"
      FL=""; case $OP in *+f) OP=${OP%+f}; FL=--openfhe-primes;; esac
      lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
      for rep in 1 2 3; do for v in "${vs[@]}"; do
        echo "$v rep$rep $(HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py $OP $FL --batch 128 --reps 20 2>/dev/null | tail -n 1)"
      done; done > "$O/abop_$OP${FL:+_f}.txt" ;;
    steptable) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/step" -o run -- python3 tools/op_bench.py ckks_mul --batch 128 --reps 8 > "$O/step.log" 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
