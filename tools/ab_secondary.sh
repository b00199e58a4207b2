#!/bin/bash
# A/B of the bench's secondary configs (C4 rotate, C3 BFV, C2 NTT) across
# library variants on ONE box.   tools/ab_secondary.sh OUT var1 var2 ...
OUT=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=herdsman_amd/lib/libherdsman_fhe.so; else lib=herdsman_amd/var/$v/libherdsman_fhe.so; fi
    HERD_FHE_LIB=$lib timeout -k 10 180 python3 bench.py --no-cpu --steps 10 > $OUT.$v.$rep.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('$OUT.$v.$rep.log').read().strip().split(chr(10))[-1]); print('$v rep$rep', d['value'], 'ct/s', d['secondary'])"
  done
done
