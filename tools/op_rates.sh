#!/bin/bash
# Per-op rates at the BASELINE configs (tools/op_bench.py), one line each, into $1/ops.txt
set -e
O=${1:-gpurun_out/ops}; mkdir -p "$O"
B=${BATCHES:-128}
for b in $B; do
  for op in ${OPS:-ckks_rot ckks_hrot bfv_mul bfv_rot bfv_hrot}; do
    echo "$(timeout -k 10 200 python3 tools/op_bench.py $op --batch $b --reps 10 | tail -n 1)"
  done
done > "$O/ops.txt"
