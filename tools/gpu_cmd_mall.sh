# FETCH/WRITE per kernel of ckks_mul, unchunked (main) vs MALL-sized chunks (tc8, cc16)
set -e
export TMPDIR=/tmp
O=gpurun_out/mall
mkdir -p $O
lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
for v in main tc8 cc16; do
  HERD_FHE_LIB=$(lib_of $v) timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$v.fetch -o run -- python3 tools/op_bench.py ckks_mul --batch 128 --reps 1 > $O/$v.fetch.log 2>&1
  HERD_FHE_LIB=$(lib_of $v) timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$v.write -o run -- python3 tools/op_bench.py ckks_mul --batch 128 --reps 1 > $O/$v.write.log 2>&1
done
