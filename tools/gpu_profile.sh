#!/bin/bash
# One gpurun call: GPU tests, default bench, kernel-trace stats, two PMC passes.
# Usage (from the repo root on the GPU box): bash tools/gpu_profile.sh TAG
set -e
TAG=${1:-r01}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- \
  python3 $R/bench.py --frames 256 --steps 3 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- \
  python3 $R/bench.py --frames 32 --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- \
  python3 $R/bench.py --frames 32 --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1
find $O -name "*.csv" | head -20
