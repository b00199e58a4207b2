# per-kernel time and bytes of the BFV C3 op (N=2^15, L=8, 128 per call)
set -e
export TMPDIR=/tmp
O=gpurun_out/bfv
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/main -o run -- python3 tools/op_bench.py bfv_mul --batch 128 --reps 5 > $O/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $O/valu -o run -- python3 tools/op_bench.py bfv_mul --batch 128 --reps 1 > $O/valu.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 tools/op_bench.py bfv_mul --batch 128 --reps 1 > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 tools/op_bench.py bfv_mul --batch 128 --reps 1 > $O/write.log 2>&1
