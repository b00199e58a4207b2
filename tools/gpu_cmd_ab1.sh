set -e
mkdir -p gpurun_out/ab1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1/gpu_main.log 2>&1
HERD_FHE_LIB=herdsman_amd/var/p1xcd/libherdsman_fhe.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_digests.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1/gpu_p1xcd.log 2>&1
HERD_FHE_LIB=herdsman_amd/var/persist2/libherdsman_fhe.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_digests.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1/gpu_persist2.log 2>&1
bash tools/ab_quick.sh gpurun_out/ab1/q main r02 persist1 persist2 xcdjob p1xcd > gpurun_out/ab1/summary.txt 2>&1
