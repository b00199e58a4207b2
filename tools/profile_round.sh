#!/bin/bash
# rocprofv3 evidence for one round (run on the GPU box):
#   1. kernel-trace + stats of the roofline-only bench (the dominant kernel group, fhe_ntt_fwd)
#   2. kernel-trace + stats of the headline on ONE stream (--streams 1: kernels do not overlap,
#      so tools/step_table.py can attribute per-wave time), 8 waves of 128
#   3. kernel stats of the 4-stream headline (2 C5 steps)
#   4. PMC passes (one counter group per run) of the roofline-only bench: FETCH_SIZE,
#      WRITE_SIZE, VALU/occupancy, instruction mix
# Usage: tools/profile_round.sh OUTDIR
set -e
OUT=${1:-gpurun_out/prof}
export TMPDIR=/tmp
mkdir -p "$OUT"
R="python3 bench.py --roofline-only --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/roofline" -o run -- \
  $R > "$OUT/roofline.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o run -- \
  python3 bench.py --steps 1 --warmup 1 --global-batch 1024 --no-cpu --no-secondary --streams 1 > "$OUT/bench.log" 2>&1
timeout -k 10 300 rocprofv3 --stats --kernel-trace --output-format csv -d "$OUT/bench4" -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu --no-secondary > "$OUT/bench4.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- $R > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- $R > "$OUT/pmc_write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d "$OUT/pmc_valu" -o run -- $R > "$OUT/pmc_valu.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS \
  SQ_LDS_BANK_CONFLICT --output-format csv -d "$OUT/pmc_mix" -o run -- $R > "$OUT/pmc_mix.log" 2>&1
echo profile passes done
# 5. per-kernel PMC account of one headline wave on one stream (tools/step_pmc.py)
S="python3 bench.py --steps 1 --warmup 1 --global-batch 128 --no-cpu --no-secondary --streams 1 --ntt-reps 1"
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES --output-format csv \
  -d "$OUT/step_valu" -o run -- $S > "$OUT/step_valu.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/step_fetch" -o run -- $S > "$OUT/step_fetch.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/step_write" -o run -- $S > "$OUT/step_write.log" 2>&1
echo step pmc done
