#!/bin/bash
# Encode A/B of library builds at F frames (each twice, interleaved), after the
# slide/route GPU tests of the in-tree build.  Usage: bash tools/gpu_abenc.sh TAG F DIR...
TAG=$1; F=$2; shift 2
export TMPDIR=/tmp; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_slide.py tests/test_classify_routes.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for d in "$@"; do
    if [ "$d" = "-" ]; then lib=""; else lib="NICE_LIB_PATH=$d/libnice_hip.so"; fi
    echo "== [$d]"; env $lib timeout -k 10 200 python tools/phase_time.py $F 3 2>&1 | grep encode || exit 1
  done
done > $O/ab.log
cat $O/ab.log
