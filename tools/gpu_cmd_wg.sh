set -e
O=${1:-gpurun_out/wg}
mkdir -p $O /tmp/wgb
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $O/nproc.txt 2>/dev/null || true; df -h /tmp >> $O/nproc.txt
timeout -k 10 400 herdsman_amd/bin/wg_run bench /tmp/wgb 0,16,12,4,3,0 4 64 4 64 5 > $O/wg_b64.txt 2>&1
timeout -k 10 400 herdsman_amd/bin/wg_run bench /tmp/wgb 0,16,12,4,3,0 4 64 4 16 5 > $O/wg_b16.txt 2>&1
WG_IO_THREADS=1 timeout -k 10 400 herdsman_amd/bin/wg_run bench /tmp/wgb 0,16,12,4,3,0 4 64 4 16 5 > $O/wg_b16_t1.txt 2>&1
WG_IO_THREADS=8 timeout -k 10 400 herdsman_amd/bin/wg_run bench /tmp/wgb 0,16,12,4,3,0 4 64 4 16 5 > $O/wg_b16_t8.txt 2>&1
timeout -k 10 400 herdsman_amd/bin/wg_run bench /tmp/wgb 0,16,12,4,3,0 8 64 8 16 5 > $O/wg_b16_l8.txt 2>&1
