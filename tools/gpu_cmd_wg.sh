set -e
O=${1:-gpurun_out/wg}
mkdir -p $O /tmp/wgb
timeout -k 10 300 python -u -m pytest tests/test_worker_group.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/wg_tests.log 2>&1
timeout -k 10 400 herdsman_amd/bin/wg_run bench /tmp/wgb 0,16,12,4,3,0 4 64 4 64 5 > $O/wg_b64.txt 2>&1
timeout -k 10 400 herdsman_amd/bin/wg_run bench /tmp/wgb 0,16,12,4,3,0 4 64 4 16 5 > $O/wg_b16.txt 2>&1
