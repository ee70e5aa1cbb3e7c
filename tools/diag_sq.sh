#!/bin/bash
# One gpurun call: decoder stats on one 4K frame, then SQ counter passes over a
# 32-frame bench step.  Usage: bash tools/diag_sq.sh TAG
set -e
TAG=${1:-diag}
R=$(pwd)
O=$R/gpurun_out/$TAG
S=/tmp/diag_$TAG
mkdir -p $O $S
export TMPDIR=/tmp
NICE_DEC_STATS=1 timeout -k 10 300 python tools/dec1.py > $O/dec1_stats.log 2>&1
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d $S/p1 -o run -- python3 $R/bench.py --frames 32 --steps 1 --warmup 1 --no-cpu-baseline > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH \
  --output-format csv -d $S/p2 -o run -- python3 $R/bench.py --frames 32 --steps 1 --warmup 1 --no-cpu-baseline > $O/p2.log 2>&1
cd $R
python3 tools/pmc_dump.py $(find $S/p1 -name "*counter_collection.csv") > $O/p1.txt
python3 tools/pmc_dump.py $(find $S/p2 -name "*counter_collection.csv") > $O/p2.txt
cat $O/dec1_stats.log $O/p1.txt $O/p2.txt
