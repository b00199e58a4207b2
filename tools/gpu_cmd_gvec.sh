# Generic-moduli butterflies in lock-step (gvec) against main: generic/all parity on gvec, paired per-op A/B
set -e
export TMPDIR=/tmp
O=gpurun_out/gvec
mkdir -p $O
lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
HERD_FHE_LIB=$(lib_of gvec) timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_digests.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests_gvec.log 2>&1
for rep in 1 2 3; do
  for v in main gvec; do
    for op in "ckks_mul --openfhe-primes" "ckks_mul"; do
      echo -n "$op $v rep$rep " >> $O/ab.txt
      HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py $op --batch 128 --reps 20 2>/dev/null | tail -n 1 >> $O/ab.txt
    done
  done
done
