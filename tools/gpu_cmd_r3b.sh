set -e
export TMPDIR=/tmp
O=${1:-gpurun_out/r3b}
mkdir -p $O /tmp/wgb
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_all.log 2>&1
bash tools/ab_quick.sh $O/q main ${BASE:-c2} > $O/ab.txt 2>&1
S="python3 bench.py --steps 1 --warmup 1 --global-batch 128 --no-cpu --no-secondary --streams 1 --ntt-reps 1"
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $O/step_valu -o run -- $S > $O/step_valu.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/step_fetch -o run -- $S > $O/step_fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/step_write -o run -- $S > $O/step_write.log 2>&1


