#!/bin/bash
# One gpurun call for scarce boxes: A/B phase times of library builds (F and 1
# frame), then the full profile of the in-tree build (tests, bench, kernel
# trace, PMC traffic).  Usage: bash tools/gpu_round.sh TAG F DIR...
TAG=$1; F=$2; shift 2
mkdir -p gpurun_out/$TAG
for d in "$@"; do
  echo "== $d $F"; NICE_LIB_PATH=$d/libnice_hip.so timeout -k 10 200 python tools/phase_time.py $F 3 2>&1 | grep -E "encode|decode" || exit 1
  echo "== $d 1"; NICE_LIB_PATH=$d/libnice_hip.so timeout -k 10 100 python tools/phase_time.py 1 3 2>&1 | grep -E "encode|decode" || exit 1
done 2>&1 | tee gpurun_out/$TAG/ab.log
bash tools/gpu_profile.sh $TAG
