#!/bin/bash
# Builds libnice_hip.so of a git revision into ab/NAME (for tools/abn.sh A/B runs).
# Usage: [EXTRA="-DFOO"] bash tools/build_ab.sh REV NAME
set -e
REV=${1:-HEAD}; NAME=${2:-head}
R=$(git rev-parse --show-toplevel)
T=$(mktemp -d /tmp/ab_XXXX)
git -C "$R" archive "$REV" fast-losless-image-compression-format_amd/csrc include | tar -x -C "$T"
cd "$T/fast-losless-image-compression-format_amd"
pids=""
for f in nice_encode nice_decode nice_capi nice_pipe nice_image; do
  [ -f csrc/$f.hip ] || continue
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function $EXTRA \
    -c csrc/$f.hip -o $T/$f.o &
  pids="$pids $!"
done
for p in $pids; do wait $p || { echo "build_ab: compile failed" >&2; rm -rf "$T"; exit 1; }; done
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -c csrc/nice_png.cpp -o $T/png.o
mkdir -p "$R/ab/$NAME"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -shared -o "$R/ab/$NAME/libnice_hip.so" $T/*.o
rm -rf "$T"
echo "built ab/$NAME from $REV"
