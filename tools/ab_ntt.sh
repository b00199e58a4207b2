#!/bin/bash
# A/B the forward-NTT roofline loop and the headline step across library
# variants on ONE box (DVFS/device spread makes cross-box comparisons useless).
#   tools/ab_ntt.sh OUT var1 var2 ...   (var "main" = herdsman_amd/lib)
OUT=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=herdsman_amd/lib/libherdsman_fhe.so; else lib=herdsman_amd/var/$v/libherdsman_fhe.so; fi
    HERD_FHE_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu --no-secondary --steps 10 > $OUT.$v.$rep.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('$OUT.$v.$rep.log').read().strip().split(chr(10))[-1]); print('$v rep$rep', d['value'], 'ct/s  ntt_ms', d['roofline']['launch_ms'], 'frac', d['roofline']['frac'])"
  done
done
