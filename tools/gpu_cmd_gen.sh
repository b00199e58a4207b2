# per-kernel time of the C5 op on the default vs OpenFHE-style primes
set -e
export TMPDIR=/tmp
O=gpurun_out/gen
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/sp -o run -- python3 tools/op_bench.py ckks_mul --batch 128 --reps 5 > $O/sp.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/gen -o run -- python3 tools/op_bench.py ckks_mul --batch 128 --reps 5 --openfhe-primes > $O/gen.log 2>&1
timeout -k 10 200 python3 tools/op_bench.py ckks_mul --batch 128 --reps 20 >> $O/sp.log 2>&1
timeout -k 10 200 python3 tools/op_bench.py ckks_mul --batch 128 --reps 20 --openfhe-primes >> $O/gen.log 2>&1
