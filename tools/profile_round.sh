#!/bin/bash
# rocprofv3 evidence for one round (run on the GPU box):
#   1. kernel-trace + stats of the roofline-only bench (the dominant kernel group, fhe_ntt_fwd)
#   2. kernel-trace + stats of the headline step on ONE stream (--streams 1: kernels do not
#      overlap, so tools/step_table.py can attribute per-step time)
#   3. FETCH_SIZE and WRITE_SIZE passes (separate runs) of the roofline-only bench
# Usage: tools/profile_round.sh OUTDIR
set -e
OUT=${1:-gpurun_out/prof}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/roofline" -o run -- \
  python3 bench.py --roofline-only --no-cpu > "$OUT/roofline.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu --no-secondary --streams 1 > "$OUT/bench.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
  python3 bench.py --roofline-only --no-cpu > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
  python3 bench.py --roofline-only --no-cpu > "$OUT/pmc_write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv \
  -d "$OUT/pmc_valu" -o run -- python3 bench.py --roofline-only --no-cpu > "$OUT/pmc_valu.log" 2>&1
echo profile done
