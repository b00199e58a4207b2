# per-kernel trace of ckks_mul per library variant + op_bench A/B
#   bash tools/gpu_cmd_kp.sh OUT var...   (var "main" = herdsman_amd/lib)
set -e
export TMPDIR=/tmp
O=$1; shift
mkdir -p $O
lib_of() { if [ "$1" = main ]; then echo herdsman_amd/lib/libherdsman_fhe.so; else echo herdsman_amd/var/$1/libherdsman_fhe.so; fi; }
for v in "$@"; do
  HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/op_bench.py ckks_mul --batch 128 --reps 5 > $O/$v.log 2>&1
done
for rep in 1 2; do
  for v in "$@"; do
    echo -n "mul $v rep$rep " >> $O/ab.txt
    HERD_FHE_LIB=$(lib_of $v) timeout -k 10 200 python3 tools/op_bench.py ckks_mul --batch 128 --reps 20 2>/dev/null | tail -n 1 >> $O/ab.txt
  done
done
