#!/bin/bash
# Register / spill / occupancy table of one translation unit's kernels at compile time
# (hipcc -Rpass-analysis=kernel-resource-usage), without building the library.
#   tools/kreg.sh csrc/ntt_conv34.hip [name-regex] [extra hipcc flags...]
set -e
cd "$(dirname "$0")/../herdsman_amd"
SRC=$1; FILT=${2:-.}; shift; shift || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../include "$@" -Rpass-analysis=kernel-resource-usage \
  -c -o /tmp/kreg.$$.o "$SRC" 2>&1 | python3 -c '
import re, sys
filt = re.compile(sys.argv[1]); cur = None; rows = {}
for ln in sys.stdin:
    m = re.search(r"Function Name: (\S+)", ln)
    if m: cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", ln)
    if cur and m: rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    if filt.search(k):
        g = lambda key: v.get(key, "?")
        print("%-90s vgpr %4s spill %4s occ %s" % (k[:90], g("VGPRs"), g("VGPRs Spill"), g("Occupancy [waves/SIMD]")))
' "$FILT"
rm -f /tmp/kreg.$$.o
