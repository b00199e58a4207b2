# GPU suite, headline quick A/B and the per-op rates (CKKS mul, rotate, BFV mul, CKKS mul on
# OpenFHE-style primes) of main against one variant, alternating
#   bash tools/gpu_cmd_full_ab.sh OUT VARIANT
set -e
export TMPDIR=/tmp
O=$1; V=$2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_all.log 2>&1
bash tools/ab_quick.sh $O/q main $V > $O/abq.txt 2>&1
lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
for rep in 1 2; do
  for v in main $V; do
    for op in "ckks_mul" "ckks_rot" "bfv_mul" "ckks_mul --openfhe-primes"; do
      echo -n "$v rep$rep " >> $O/ab.txt
      HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py $op --batch 128 --reps 20 2>/dev/null | tail -n 1 | sed "s/^/$op: /" >> $O/ab.txt
    done
  done
done
