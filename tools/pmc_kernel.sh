#!/bin/bash
# SQ counter passes for one bench step of F frames; prints the counters of the
# kernels matching PATTERN (last dispatch each).  Usage: bash tools/pmc_kernel.sh TAG F PATTERN
set -e
TAG=${1:-pmc}; F=${2:-32}; PAT=${3:-nice::}
R=$(pwd); O=$R/gpurun_out/$TAG; S=/tmp/pmc_$TAG
mkdir -p $O $S
export TMPDIR=/tmp
cd /tmp
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "nice::" --output-format csv -d $S/p$i -o run -- \
    python3 $R/tools/phase_time.py $F 1 > $O/p$i.log 2>&1
  python3 $R/tools/pmc_dump.py $(find $S/p$i -name "*counter_collection.csv") | grep "$PAT" > $O/p$i.txt || true
done
cat $O/p*.txt
