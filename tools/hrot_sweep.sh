#!/bin/bash
# hoisted-rotation rates over batch size and rotations per call (tools/op_bench.py ckks_hrot)
set -e
O=${1:-gpurun_out/hrot}; mkdir -p "$O"
for b in 1 4 16; do for r in 1 4 8 16; do
  echo "batch $b rot $r: $(timeout -k 10 200 python3 tools/op_bench.py ckks_hrot --batch $b --rot $r --reps 10 | tail -n 1)"
done; done > "$O/hrot.txt"
for b in 1 4 16; do echo "batch $b plain: $(timeout -k 10 200 python3 tools/op_bench.py ckks_rot --batch $b --reps 10 | tail -n 1)"; done >> "$O/hrot.txt"
