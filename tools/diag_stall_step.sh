#!/bin/bash
# Stall counters of every kernel of one 1-stream headline wave (tools/diag_stall.sh's
# counter groups, one group per run).   Usage: tools/diag_stall_step.sh OUTDIR [COMMAND]
# (COMMAND: another workload, e.g. "python3 tools/op_bench.py bfv_mul --batch 128 --reps 1")
set -e
OUT=${1:-gpurun_out/stallstep}
export TMPDIR=/tmp
mkdir -p "$OUT"
S=${2:-"python3 bench.py --steps 1 --warmup 1 --global-batch 128 --no-cpu --no-secondary --streams 1 --ntt-reps 1"}
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "TA_BUSY_avr TA_TA_BUSY_sum" \
           "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- $S > "$OUT/p$i.log" 2>&1
done
echo stall passes done
