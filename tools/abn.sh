#!/bin/bash
# Encode/decode phase times of several library builds: bash tools/abn.sh F DIR...
F=$1; shift
for d in "$@"; do
  echo "== $d"; NICE_LIB_PATH=$d/libnice_hip.so timeout -k 10 200 python tools/phase_time.py $F 3 || exit 1
done
