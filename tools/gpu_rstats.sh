#!/bin/bash
# Row-kernel cycle split (NICE_ROWS_STATS build in ab/rstats): one 4K frame and
# one 1920x1080 frame.  Usage: bash tools/gpu_rstats.sh TAG
TAG=${1:-rstats}; O=gpurun_out/$TAG; mkdir -p $O
NICE_LIB_PATH=ab/rstats/libnice_hip.so NICE_DEC_STATS=1 timeout -k 10 200 python tools/dec1.py > $O/dec1_4k.log 2>&1 || exit 1
W=1920 H=1080 NICE_LIB_PATH=ab/rstats/libnice_hip.so NICE_DEC_STATS=1 timeout -k 10 200 python tools/dec1.py > $O/dec1_1080p.log 2>&1 || exit 1
grep -h "stats\|ok" $O/dec1_4k.log $O/dec1_1080p.log
