#!/bin/bash
# One gpurun call: GPU tests, default bench, kernel-trace stats, two PMC passes.
# Usage (from the repo root on the GPU box): bash tools/gpu_profile.sh TAG [FRAMES]
set -e
TAG=${1:-r01}
FR=${2:-512}
R=$(pwd)
O=$R/gpurun_out/$TAG
S=/tmp/prof_$TAG
mkdir -p $O $S
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then   # (tools/gpu_r04.sh runs them first)
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  tail -2 $O/pytest_gpu.log
fi
timeout -k 10 400 python bench.py --frames $FR > $O/bench.json 2> $O/bench.err
cat $O/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $S/kt -o run -- \
  python3 $R/bench.py --frames $FR --steps 3 --warmup 1 --no-cpu-baseline --streamed-frames 0 > $O/kt.log 2>&1
# counter passes: every dispatch encodes or decodes the same 32 frames (no
# single-frame or config-4 dispatches in the per-kernel averages)
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "nice::" --output-format csv -d $S/pmc_fetch -o run -- \
  python3 $R/tools/phase_time.py 32 1 > $O/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "nice::" --output-format csv -d $S/pmc_write -o run -- \
  python3 $R/tools/phase_time.py 32 1 > $O/pmc_write.log 2>&1
cd $R
find $S -name "*.csv" -exec ls -la {} \; > $O/files.txt
cp $(find $S/kt -name "*kernel_stats.csv") $O/kernel_stats.csv
python3 tools/pmc_traffic.py 32 $(find $S/pmc_fetch -name "*counter_collection.csv") \
  $(find $S/pmc_write -name "*counter_collection.csv") > $O/pmc_traffic.json
cat $O/kernel_stats.csv | cut -c1-200
cat $O/pmc_traffic.json
