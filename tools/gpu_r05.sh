#!/bin/bash
# One gpurun call: the GPU tests of the in-tree build, then A/B phase times at
# F frames and at one frame of the builds/environments given.
# Usage: bash tools/gpu_r05.sh TAG F [tests] -- "DIR|ENV" ...
#   DIR: a build directory (ab/NAME) with the in-tree environment; ENV: "VAR=1 ..."
#   for the in-tree build ("-": none).
TAG=$1; F=$2; shift 2
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
if [ "$1" != "--" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
  shift
fi
shift
for e in "$@"; do
  if [ -d "$e" ]; then lib="NICE_LIB_PATH=$e/libnice_hip.so"; env=""; else lib=""; env="$e"; [ "$e" = "-" ] && env=""; fi
  echo "== [$e] $F"; env $lib $env timeout -k 10 200 python tools/phase_time.py $F 3 || exit 1
  echo "== [$e] 1"; env $lib $env timeout -k 10 100 python tools/phase_time.py 1 3 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
