# Round-3 final tree (column-sum conversions in main): full GPU suite, smoke, default bench line (with the CPU baseline)
set -e
export TMPDIR=/tmp
O=gpurun_out/final3
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1
