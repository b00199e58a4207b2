# per-kernel trace of the metric op (op_bench ckks_mul, 128 per call) on the default special primes
# and on OpenFHE-style generic primes, one box: where the generic product's time goes
set -e
export TMPDIR=/tmp
O=${1:-gpurun_out/gen}; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sp -o run -- python3 tools/op_bench.py ckks_mul --batch 128 --reps 5 > $O/sp.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gen -o run -- python3 tools/op_bench.py ckks_mul --batch 128 --reps 5 --openfhe-primes > $O/gen.log 2>&1
for v in sp gen; do f=$(find $O/$v -name run_kernel_stats.csv | head -n 1); [ "$f" = $O/$v/run_kernel_stats.csv ] || cp "$f" $O/$v/run_kernel_stats.csv; done
python3 tools/kstat_cmp.py $O sp gen > $O/kcmp.txt
