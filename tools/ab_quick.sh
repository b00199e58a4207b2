#!/bin/bash
# Quick A/B of library variants on ONE box: the N=2^16 NTT passes (tools/ntt_bench.py,
# 4608 limbs = one wave's ModUp) and the headline (bench.py, 3 steps of the C5 batch).
#   tools/ab_quick.sh OUT var1 var2 ...   (var "main" = herdsman_amd/lib)
OUT=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=herdsman_amd/lib/libherdsman_fhe.so; else lib=herdsman_amd/var/$v/libherdsman_fhe.so; fi
    HERD_FHE_LIB=$lib timeout -k 10 120 python3 tools/ntt_bench.py --log-n 16 --limbs 4608 > $OUT.$v.$rep.ntt 2>&1 || exit 1
    HERD_FHE_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --no-secondary --steps 3 --warmup 1 > $OUT.$v.$rep.log 2>&1 || exit 1
    echo "$v rep$rep: $(grep -o 'fwd: [0-9.]* ms\|inv: [0-9.]* ms' $OUT.$v.$rep.ntt | tr '\n' ' ') $(python3 -c "import json; d=json.loads(open('$OUT.$v.$rep.log').read().strip().split(chr(10))[-1]); print('headline', d['value'], 'ct/s frac', d['roofline']['frac'])")"
  done
done
