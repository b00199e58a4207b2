# paired A/B of library variants on one box: tools/gpu_cmd_ab.sh OUT var...
set -e
export TMPDIR=/tmp
O=$1; shift
mkdir -p $O
bash tools/ab_quick.sh $O/q "$@" > $O/ab.txt 2>&1
