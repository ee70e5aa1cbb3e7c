#!/bin/bash
# PMC traffic passes only (FETCH_SIZE, WRITE_SIZE) over 32-frame dispatches.
# Usage (repo root on the GPU box): bash tools/pmc_only.sh TAG
set -e
TAG=${1:-pmc}
R=$(pwd); O=$R/gpurun_out/$TAG; S=/tmp/prof_$TAG
mkdir -p $O $S
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "nice::" --output-format csv -d $S/pmc_fetch -o run -- \
  python3 $R/tools/phase_time.py 32 1 > $O/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "nice::" --output-format csv -d $S/pmc_write -o run -- \
  python3 $R/tools/phase_time.py 32 1 > $O/pmc_write.log 2>&1
cd $R
python3 tools/pmc_traffic.py 32 $(find $S/pmc_fetch -name "*counter_collection.csv") \
  $(find $S/pmc_write -name "*counter_collection.csv") > $O/pmc_traffic.json
cat $O/pmc_traffic.json
