# GPU suite, then the quick headline A/B of main against the given variants
#   bash tools/gpu_cmd_suite_ab.sh OUT var...
set -e
export TMPDIR=/tmp
O=$1; shift
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_all.log 2>&1
bash tools/ab_quick.sh $O/q main "$@" > $O/abq.txt 2>&1
