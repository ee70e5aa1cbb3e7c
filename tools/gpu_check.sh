#!/bin/bash
# One gpurun call: the GPU test suite, then the default bench line.
# Usage (repo root on the GPU box): bash tools/gpu_check.sh TAG [bench args...]
set -e
TAG=${1:-chk}; shift || true
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
