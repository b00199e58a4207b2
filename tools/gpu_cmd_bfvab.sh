# GPU suite, then BFV C3 op A/B (main vs the given variant) and its kernel times
set -e
export TMPDIR=/tmp
O=$1; V=$2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_all.log 2>&1
lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
for rep in 1 2 3; do
  for v in main $V; do
    echo -n "bfv $v rep$rep " >> $O/ab.txt
    HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py bfv_mul --batch 128 --reps 20 2>/dev/null | tail -n 1 >> $O/ab.txt
  done
done
for v in main $V; do
  HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/op_bench.py bfv_mul --batch 128 --reps 5 > $O/$v.log 2>&1
done
