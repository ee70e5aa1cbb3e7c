#!/bin/bash
# One gpurun call: the GPU tests (stop at the first failure), then a short bench.
# Usage (repo root on the GPU box): bash tools/gpu_quick.sh TAG [bench args...]
TAG=${1:-q}; shift || true
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -15 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
