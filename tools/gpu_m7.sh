# one-off (round 6): parity of library variants, then a paired BFV A/B
set -e
O=${1:-gpurun_out/m8}; shift || true; mkdir -p $O
VS=${VS:-pf lsw4 pflsw4}
OP=${OP:-bfv_mul}
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bfv or digest or behz or hps" > $O/tests_main.log 2>&1
for v in $VS; do
  HERD_FHE_LIB=herdsman_amd/var/$v/libherdsman_fhe.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bfv or digest" > $O/tests_$v.log 2>&1
done
bash tools/gpu_steps.sh $O "abop=$OP:main,${VS// /,}" optrace=$OP
