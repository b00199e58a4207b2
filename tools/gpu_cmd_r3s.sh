# Column-sum conversion variant (cols2: PRO_CONV both moduli classes + BEHZ): GPU suite on it, smoke, paired A/B with secondaries
set -e
export TMPDIR=/tmp
O=gpurun_out/r3s
mkdir -p $O
HERD_FHE_LIB=herdsman_amd/var/cols2/libherdsman_fhe.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests_cols2.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
for rep in 1 2; do
  for v in main cols2; do
    if [ "$v" = main ]; then lib=herdsman_amd/lib/libherdsman_fhe.so; else lib=herdsman_amd/var/$v/libherdsman_fhe.so; fi
    HERD_FHE_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --steps 3 --warmup 1 > $O/ab.$v.$rep.log 2>&1
    python3 -c "import json; d=json.loads(open('$O/ab.$v.$rep.log').read().strip().split(chr(10))[-1]); print('$v', $rep, d['value'], d['secondary'])" >> $O/ab.txt
  done
done
