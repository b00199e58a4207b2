#!/bin/bash
# Build a variant of the backend library into herdsman_amd/var/<name>/ from a
# patched copy of csrc (for A/B runs: HERD_FHE_LIB=herdsman_amd/var/<name>/libherdsman_fhe.so).
#   tools/build_variant.sh NAME [sed-expression FILE]...
#   REV=<git rev> tools/build_variant.sh NAME ...   (csrc taken from that revision)
#   EXTRA='<hipcc flags>' tools/build_variant.sh NAME  (extra flags for the .hip translation units)
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/herdsman_amd/var/$NAME
rm -rf "$D"; mkdir -p "$D/csrc"
if [ -n "$REV" ]; then
  # the source list of that revision (files were added and split between rounds)
  for f in $(git -C "$ROOT" ls-tree --name-only "$REV" herdsman_amd/csrc/); do
    git -C "$ROOT" show "$REV:$f" > "$D/csrc/$(basename "$f")"
  done
else
  cp "$ROOT"/herdsman_amd/csrc/* "$D/csrc/"
fi
sed -i "s@\"../../include/plugins/fhe_backend.h\"@\"plugins/fhe_backend.h\"@" "$D"/csrc/*.hpp "$D"/csrc/*.cpp "$D"/csrc/*.hip
while [ $# -ge 2 ]; do sed -i "$1" "$D/csrc/$2"; shift 2; done
cd "$D"
for f in csrc/*.hip; do b=$(basename "$f" .hip); /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$ROOT/include" $EXTRA -c -o $b.o "$f" & done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$ROOT/include" -x hip -c -o be.o csrc/fhe_backend.cpp &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o libherdsman_fhe.so *.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f *.o
echo "built $D/libherdsman_fhe.so"
