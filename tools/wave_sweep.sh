#!/bin/bash
# Headline throughput vs wave geometry (ct-mults per wave, concurrent contexts):
# smaller per-context batches shrink the pipeline's working set toward the
# MALL.   tools/wave_sweep.sh OUT "batch:streams" ...
OUT=$1; shift
for cfg in "$@"; do
  b=${cfg%%:*}; s=${cfg##*:}
  timeout -k 10 120 python3 bench.py --no-cpu --no-secondary --steps 3 --warmup 1 --batch $b --streams $s > $OUT.$b.$s.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$OUT.$b.$s.log').read().strip().split(chr(10))[-1]); print('batch $b streams $s:', d['value'], 'ct/s')"
done
