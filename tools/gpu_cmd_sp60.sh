# Conversion column sums reduced in place (sp60, special targets < 2^60) against main: parity, per-kernel trace, paired A/B
set -e
export TMPDIR=/tmp
O=gpurun_out/sp60
mkdir -p $O
lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
HERD_FHE_LIB=$(lib_of sp60) timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_digests.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests_sp60.log 2>&1
for v in main sp60; do
  HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/op_bench.py ckks_mul --batch 128 --reps 5 > $O/$v.log 2>&1
done
for rep in 1 2 3; do
  for v in main sp60; do
    echo -n "ckks_mul $v rep$rep " >> $O/ab.txt
    HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py ckks_mul --batch 128 --reps 20 2>/dev/null | tail -n 1 >> $O/ab.txt
  done
done
for rep in 1 2; do
  for v in main sp60; do
    HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 bench.py --no-cpu --no-secondary --steps 3 --warmup 1 > $O/b.$v.$rep.log 2>&1
    python3 -c "import json; d=json.loads(open('$O/b.$v.$rep.log').read().strip().split(chr(10))[-1]); print('headline $v rep$rep', d['value'])" >> $O/ab.txt
  done
done
