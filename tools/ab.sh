#!/bin/bash
# A/B timing on the GPU box: phase times of the old library (ab/old) and the
# current build for F frames.  Usage: bash tools/ab.sh F [reps]
F=${1:-64}; R=${2:-3}
echo "== old"; NICE_LIB_PATH=ab/old/libnice_hip.so timeout -k 10 200 python tools/phase_time.py $F $R || exit 1
echo "== new"; timeout -k 10 200 python tools/phase_time.py $F $R
