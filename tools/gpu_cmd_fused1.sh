set -e
mkdir -p gpurun_out/f1
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 60 --timeout-method thread -k "ntt" > gpurun_out/f1/ntt_tests.log 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f1/gpu_all.log 2>&1
for A in 1 2 3 4; do HERD_NTT_FUSED_AHEAD=$A timeout -k 10 60 python3 tools/ntt_bench.py --log-n 15 16 17 --limbs 4608 > gpurun_out/f1/ntt_fused_a$A.txt 2>&1; done
HERD_NTT_FUSED=0 timeout -k 10 60 python3 tools/ntt_bench.py --log-n 15 16 17 --limbs 4608 > gpurun_out/f1/ntt_twopass.txt 2>&1
HERD_NTT_FUSED=0 timeout -k 10 120 python3 bench.py --no-cpu --no-secondary --steps 5 > gpurun_out/f1/bench_twopass.json 2>&1
timeout -k 10 120 python3 bench.py --no-cpu --no-secondary --steps 5 > gpurun_out/f1/bench_fused.json 2>&1
