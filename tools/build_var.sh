#!/bin/bash
# Builds libnice_hip.so of the WORKING TREE with extra compiler flags into
# ab/NAME (A/B variants selected by -D macros).  Usage: bash tools/build_var.sh NAME "-DFOO"
set -e
NAME=$1; FLAGS=$2
R=$(git rev-parse --show-toplevel)
T=$(mktemp -d /tmp/var_XXXX)
cd "$R/fast-losless-image-compression-format_amd"
pids=""
for f in nice_encode nice_decode nice_capi nice_pipe nice_image; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function $FLAGS \
    -c csrc/$f.hip -o $T/$f.o &
  pids="$pids $!"
done
for p in $pids; do wait $p || { echo "build_var: compile failed" >&2; rm -rf "$T"; exit 1; }; done
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -c csrc/nice_png.cpp -o $T/png.o
mkdir -p "$R/ab/$NAME"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -shared -o "$R/ab/$NAME/libnice_hip.so" $T/*.o
rm -rf "$T"
echo "built ab/$NAME ($FLAGS)"
