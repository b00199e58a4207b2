set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/f2
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 60 --timeout-method thread -k "ntt" > gpurun_out/f2/ntt_tests.log 2>&1
timeout -k 10 60 python3 tools/ntt_bench.py --log-n 15 16 17 --limbs 4608 > gpurun_out/f2/ntt_fused.txt 2>&1
HERD_NTT_FUSED=0 timeout -k 10 60 python3 tools/ntt_bench.py --log-n 15 16 17 --limbs 4608 > gpurun_out/f2/ntt_twopass.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f2/fetch -o run -- python3 tools/ntt_bench.py --log-n 16 --limbs 4608 --reps 5 > gpurun_out/f2/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/f2/write -o run -- python3 tools/ntt_bench.py --log-n 16 --limbs 4608 --reps 5 > gpurun_out/f2/write.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/f2/tcc -o run -- python3 tools/ntt_bench.py --log-n 16 --limbs 4608 --reps 5 > gpurun_out/f2/tcc.log 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f2/gpu_all.log 2>&1
