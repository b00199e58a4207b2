#!/bin/bash
# double-hoisted rotation sums against hoisted rotations (tools/op_bench.py), rates in rotations/s
set -e
O=${1:-gpurun_out/rsum}; mkdir -p "$O"
for b in 1 16 128; do for r in 4 16; do
  echo "batch $b rot $r: $(timeout -k 10 200 python3 tools/op_bench.py ckks_rsum --batch $b --rot $r --reps 10 | tail -n 1)"
  echo "batch $b rot $r: $(timeout -k 10 200 python3 tools/op_bench.py ckks_hrot --batch $b --rot $r --reps 10 | tail -n 1)"
done; done > "$O/rsum.txt"
for r in 4 16; do
  echo "bfv batch 16 rot $r: $(timeout -k 10 200 python3 tools/op_bench.py bfv_rsum --batch 16 --rot $r --reps 10 | tail -n 1)"
  echo "bfv batch 16 rot $r: $(timeout -k 10 200 python3 tools/op_bench.py bfv_hrot --batch 16 --rot $r --reps 10 | tail -n 1)"
done >> "$O/rsum.txt"
