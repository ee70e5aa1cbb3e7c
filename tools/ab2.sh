#!/bin/bash
# A/B phase times: the in-tree library against ab/NAME builds, F frames and 1.
# Usage (repo root on the GPU box): bash tools/ab2.sh F NAME...
F=$1; shift
for d in "" "$@"; do
  lib=${d:+ab/$d/libnice_hip.so}
  echo "== ${d:-tree} $F"; NICE_LIB_PATH=$lib timeout -k 10 200 python tools/phase_time.py $F 3 || exit 1
  echo "== ${d:-tree} 1"; NICE_LIB_PATH=$lib timeout -k 10 100 python tools/phase_time.py 1 3 || exit 1
done
