#!/bin/bash
# One gpurun call: the GPU tests first (stop on a failure), then A/B phase times
# of library builds (F frames and one frame), then the full profile of the
# in-tree build.  Usage: bash tools/gpu_r04.sh TAG F DIR...
TAG=$1; F=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for d in "$@"; do
  echo "== $d $F"; NICE_LIB_PATH=$d/libnice_hip.so timeout -k 10 200 python tools/phase_time.py $F 3 2>&1 | grep -E "encode|decode" || exit 1
  echo "== $d 1"; NICE_LIB_PATH=$d/libnice_hip.so timeout -k 10 100 python tools/phase_time.py 1 3 2>&1 | grep -E "encode|decode" || exit 1
done 2>&1 | tee $O/ab.log
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
[ -n "$NO_PROFILE" ] && exit 0
SKIP_TESTS=1 bash tools/gpu_profile.sh $TAG
