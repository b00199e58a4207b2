#!/bin/bash
# A/B of bench.py command-line variants on ONE box (same library):
#   tools/ab_flags.sh OUT "name:flags" ...     e.g. "stagger:" "nostagger:--no-stagger"
OUT=$1; shift
for rep in 1 2 3; do
  for v in "$@"; do
    name=${v%%:*}; flags=${v#*:}
    timeout -k 10 120 python3 bench.py --no-cpu --no-secondary --steps 10 $flags > $OUT.$name.$rep.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('$OUT.$name.$rep.log').read().strip().split(chr(10))[-1]); print('$name rep$rep', d['value'], 'ct/s')"
  done
done
