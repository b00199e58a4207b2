set -e
export TMPDIR=/tmp
O=gpurun_out/r4o; mkdir -p $O
for v in main bfvnofuse; do
  if [ $v = main ]; then L=herdsman_amd/lib/libherdsman_fhe.so; else L=herdsman_amd/var/$v/libherdsman_fhe.so; fi
  HERD_FHE_LIB=$L timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$v/fetch -o run -- python3 tools/op_bench.py bfv_mul --batch 128 --reps 2 > $O/$v.fetch.log 2>&1
  HERD_FHE_LIB=$L timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$v/write -o run -- python3 tools/op_bench.py bfv_mul --batch 128 --reps 2 > $O/$v.write.log 2>&1
done
for rep in 1 2 3; do for v in main bfvnofuse; do
  if [ $v = main ]; then L=herdsman_amd/lib/libherdsman_fhe.so; else L=herdsman_amd/var/$v/libherdsman_fhe.so; fi
  echo "$v rep$rep $(HERD_FHE_LIB=$L timeout -k 10 200 python3 tools/op_bench.py bfv_mul --batch 128 --reps 20 2>/dev/null | tail -n 1)"
done; done > $O/ab.txt
