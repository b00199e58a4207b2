set -e
O=gpurun_out/r4h; mkdir -p $O
for op in ckks_rot ckks_hrot bfv_mul bfv_rot bfv_hrot; do
  echo "$(timeout -k 10 200 python3 tools/op_bench.py $op --batch 128 --reps 10 | tail -n 1)"
done > $O/ops.txt
