#!/bin/bash
# hoisted linear transforms (tools/op_bench.py ckks_lin), rates in plaintext-weighted rotations/s
set -e
O=${1:-gpurun_out/lin}; mkdir -p "$O"
for b in 1 16 128; do
  echo "batch $b rot 16: $(timeout -k 10 200 python3 tools/op_bench.py ckks_lin --batch $b --rot 16 --reps 10 | tail -n 1)"
done > "$O/lin.txt"
