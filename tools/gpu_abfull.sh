#!/bin/bash
# One GPU call: the whole GPU test suite, then encode + decode phase times of
# the working tree and ab/ builds, alternating (512 x 4K, one 4K frame,
# 64 x 1080p; every run checks the decoded frames).  Usage: bash tools/gpu_abfull.sh TAG DIR...
export TMPDIR=/tmp; TAG=$1; shift; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for d in - "$@"; do
  if [ "$d" = "-" ]; then lib=""; else lib="NICE_LIB_PATH=$d/libnice_hip.so"; fi
  for sh in "512 3" "1 5" "64 3 1920 1080"; do echo "== [$d] $sh"; env $lib timeout -k 10 200 python tools/phase_time.py $sh 2>&1 | grep -E "encode|decode|Error|assert" || exit 1; done
done; done > $O/ab.log
cat $O/ab.log
