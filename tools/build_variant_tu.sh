#!/bin/bash
# A library variant that differs from the main build in ONE translation unit
# (herdsman_amd/var/<name>/libherdsman_fhe.so): the TU is recompiled from a
# patched copy of csrc, every other object is the main build's (the headers
# must be unchanged).  Seconds instead of tools/build_variant.sh's full rebuild.
#   tools/build_variant_tu.sh NAME TU.hip [sed-expression FILE]...
set -e
NAME=$1; TU=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/herdsman_amd/var/$NAME
rm -rf "$D"; mkdir -p "$D/csrc"
cp "$ROOT"/herdsman_amd/csrc/* "$D/csrc/"
sed -i "s@\"../../include/plugins/fhe_backend.h\"@\"plugins/fhe_backend.h\"@" "$D"/csrc/*.hpp "$D"/csrc/*.cpp "$D"/csrc/*.hip
while [ $# -ge 2 ]; do sed -i "$1" "$D/csrc/$2"; shift 2; done
cd "$D"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$ROOT/include" $EXTRA -c -o tu.o "csrc/$TU"
objs=""
for o in "$ROOT"/herdsman_amd/build/*.o; do
  [ "$(basename "$o")" = "$TU.o" ] || objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o libherdsman_fhe.so tu.o $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f tu.o
echo "built $D/libherdsman_fhe.so ($TU patched)"
