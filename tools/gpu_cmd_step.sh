# Per-kernel account of one headline wave (1 stream): kernel trace + PMC passes
#   bash tools/gpu_cmd_step.sh OUT
set -e
export TMPDIR=/tmp
O=${1:-gpurun_out/step}
mkdir -p $O
S="python3 bench.py --steps 1 --warmup 1 --global-batch 128 --no-cpu --no-secondary --streams 1 --ntt-reps 1"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $S > $O/trace.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $O/valu -o run -- $S > $O/valu.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $S > $O/fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $S > $O/write.log 2>&1
