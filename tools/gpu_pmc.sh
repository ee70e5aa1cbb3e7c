#!/bin/bash
# PMC passes only (HBM traffic: FETCH_SIZE / WRITE_SIZE; SQ counters), every
# dispatch 32 frames, with the 512-frame bench's row kernel (dec_rows_flow
# with one row group: NICE_DEC_FLOW=1; 32 frames alone would take two).
# Usage: bash tools/gpu_pmc.sh TAG
set -e
TAG=${1:-pmc}
R=$(pwd); O=$R/gpurun_out/$TAG; S=/tmp/prof_$TAG
mkdir -p $O $S
export TMPDIR=/tmp NICE_DEC_FLOW=1
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "nice::" --output-format csv -d $S/pmc_fetch -o run -- \
  python3 $R/tools/phase_time.py 32 1 > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "nice::" --output-format csv -d $S/pmc_write -o run -- \
  python3 $R/tools/phase_time.py 32 1 > $O/pmc_write.log 2>&1
cd $R
python3 tools/pmc_traffic.py 32 $(find $S/pmc_fetch -name "*counter_collection.csv") \
  $(find $S/pmc_write -name "*counter_collection.csv") > $O/pmc_traffic.json
bash tools/pmc_kernel.sh ${TAG}_sq 32 "nice::" > $O/pmc_sq.txt
