set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/f3
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 60 --timeout-method thread -k "ntt" > gpurun_out/f3/ntt_tests.log 2>&1
for v in main fst1 fst2; do
  if [ $v = main ]; then lib=herdsman_amd/lib/libherdsman_fhe.so; else lib=herdsman_amd/var/$v/libherdsman_fhe.so; fi
  HERD_FHE_LIB=$lib timeout -k 10 60 python3 tools/ntt_bench.py --log-n 15 16 17 --limbs 4608 > gpurun_out/f3/ntt_$v.txt 2>&1
  HERD_FHE_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f3/fetch_$v -o run -- python3 tools/ntt_bench.py --log-n 16 --limbs 4608 --reps 5 > gpurun_out/f3/fetch_$v.log 2>&1
  HERD_FHE_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/f3/write_$v -o run -- python3 tools/ntt_bench.py --log-n 16 --limbs 4608 --reps 5 > gpurun_out/f3/write_$v.log 2>&1
done
HERD_NTT_FUSED=0 timeout -k 10 60 python3 tools/ntt_bench.py --log-n 15 16 17 --limbs 4608 > gpurun_out/f3/ntt_twopass.txt 2>&1
