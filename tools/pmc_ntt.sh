#!/bin/bash
# PMC passes over the N=2^16 NTT micro-benchmark (run on the GPU box).
# Usage: tools/pmc_ntt.sh OUTDIR [extra args to ntt_bench.py]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- python3 tools/ntt_bench.py --log-n 16 --reps 5 "$@" > "$OUT/p$i.log" 2>&1
done
echo done
