# generic-modulus reduction and folded BEHZ constants: parity suite, then
# op_bench A/Bs (generic primes: main vs gen0; BFV C3: main vs head)
set -e
export TMPDIR=/tmp
O=gpurun_out/gen2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_all.log 2>&1
lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
for rep in 1 2 3; do
  for v in main gen0; do
    echo -n "generic $v rep$rep " >> $O/ab.txt
    HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py ckks_mul --batch 128 --reps 20 --openfhe-primes 2>/dev/null | tail -n 1 >> $O/ab.txt
  done
  for v in main head; do
    echo -n "bfv $v rep$rep " >> $O/ab.txt
    HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py bfv_mul --batch 128 --reps 20 2>/dev/null | tail -n 1 >> $O/ab.txt
  done
done
