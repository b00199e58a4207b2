# P-limb inner product inside INTT(acc_P): GPU suite, then headline + rotate A/B (main vs ksp0)
set -e
export TMPDIR=/tmp
O=gpurun_out/ksp
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_all.log 2>&1
lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
for rep in 1 2 3; do
  for v in main ksp0; do
    echo -n "rot $v rep$rep " >> $O/ab.txt
    HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py ckks_rot --batch 128 --reps 20 2>/dev/null | tail -n 1 >> $O/ab.txt
    echo -n "mul $v rep$rep " >> $O/ab.txt
    HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py ckks_mul --batch 128 --reps 20 2>/dev/null | tail -n 1 >> $O/ab.txt
  done
done
bash tools/ab_quick.sh $O/q main ksp0 > $O/abq.txt 2>&1
