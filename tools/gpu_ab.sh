#!/bin/bash
# A/B phase times: bash tools/gpu_ab.sh TAG "F [W H]" "ENV|DIR" ...  (after the GPU tests when TESTS=1)
TAG=$1; SHAPE=$2; shift 2
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
set -- "$@"
for e in "$@"; do
  if [ -d "$e" ]; then lib="NICE_LIB_PATH=$e/libnice_hip.so"; env=""; else lib=""; env="$e"; [ "$e" = "-" ] && env=""; fi
  for sh in $SHAPE; do
    sh=${sh//,/ }
    echo "== [$e] $sh"; env $lib $env timeout -k 10 200 python tools/phase_time.py $sh || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.log
