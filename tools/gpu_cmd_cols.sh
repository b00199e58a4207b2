# Column-sum conversions: per-kernel trace of one 128-ct CKKS mul+relin and BFV mul+relin per library
# (main = column sums, base = round-3 library), then paired op-rate A/B incl. OpenFHE-style primes
set -e
export TMPDIR=/tmp
O=gpurun_out/cols
mkdir -p $O
lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
for v in main base; do
  HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/op_bench.py ckks_mul --batch 128 --reps 5 > $O/$v.log 2>&1
  HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bfv_$v -o run -- python3 tools/op_bench.py bfv_mul --batch 128 --reps 5 > $O/bfv_$v.log 2>&1
done
for rep in 1 2 3; do
  for v in main base; do
    for op in "ckks_mul" "ckks_mul --openfhe-primes" "bfv_mul"; do
      echo -n "$op $v rep$rep " >> $O/ab.txt
      HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py $op --batch 128 --reps 20 2>/dev/null | tail -n 1 >> $O/ab.txt
    done
  done
done
