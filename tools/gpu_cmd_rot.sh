# rotation reads sigma_g(c0) in the combine epilogue: GPU suite, then C4 A/B (main vs head)
set -e
export TMPDIR=/tmp
O=gpurun_out/rot
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_all.log 2>&1
lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
for rep in 1 2 3; do
  for v in main head; do
    echo -n "rot $v rep$rep " >> $O/ab.txt
    HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py ckks_rot --batch 128 --reps 20 2>/dev/null | tail -n 1 >> $O/ab.txt
  done
done
bash tools/ab_quick.sh $O/q main head > $O/abq.txt 2>&1
