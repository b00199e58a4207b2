# A/B: KSQ prefetch depth (pd3, bip2) and the pipelined automorphism (aut2)
set -e
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
bash tools/ab_quick.sh $O/q main pd3 bip2 > $O/ab.txt 2>&1
for v in main aut2; do
  if [ "$v" = main ]; then lib=herdsman_amd/lib/libherdsman_fhe.so; else lib=herdsman_amd/var/$v/libherdsman_fhe.so; fi
  HERD_FHE_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu --steps 3 --warmup 1 > $O/sec.$v.log 2>&1
done
