#!/bin/bash
# One gpurun call: selected GPU tests (pytest -k EXPR, "" = all), then phase
# times of several library builds.  Usage: bash tools/gpu_ab.sh TAG "K_EXPR" F DIR...
TAG=$1; K=$2; F=$3; shift 3
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && { tail -40 $O/pytest_gpu.log; exit $rc; }
fi
for d in "$@"; do
  echo "== $d $F"; NICE_LIB_PATH=$d/libnice_hip.so timeout -k 10 200 python tools/phase_time.py $F 3 || exit 1
  echo "== $d 1"; NICE_LIB_PATH=$d/libnice_hip.so timeout -k 10 100 python tools/phase_time.py 1 3 || exit 1
done 2>&1 | tee $O/ab.log
