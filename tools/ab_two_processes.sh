#!/bin/bash
for rep in 1 2; do
  timeout -k 10 120 python3 bench.py --no-cpu --no-secondary --steps 10 > gpurun_out/tp1.$rep.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/tp1.$rep.log').read().strip().split(chr(10))[-1]); print('1proc rep$rep', d['value'])"
  HERD_BENCH_DIST=gloo timeout -k 10 180 python3 bench.py --gpus 2 --no-cpu --no-secondary --steps 10 > gpurun_out/tp2.$rep.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/tp2.$rep.log').read().strip().split(chr(10))[-1]); print('2proc rep$rep', d['value'], d['per_rank_ct_mult_per_s'])"
done
