#!/bin/bash
# One GPU call of round 6: the GPU tests (optionally a -k filter), then phase
# times of the in-tree build at F frames and one frame.
# Usage: bash tools/gpu_r06.sh TAG [F] [PYTEST_K]
TAG=$1; F=${2:-512}; K=$3
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/pytest_gpu.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1
fi
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/phase_time.py $F 3 > $O/phase.log 2>&1 || exit 1
timeout -k 10 200 python tools/phase_time.py 1 5 >> $O/phase.log 2>&1 || exit 1
cat $O/phase.log | grep -v amdgpu.ids
