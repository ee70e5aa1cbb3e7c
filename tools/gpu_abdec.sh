#!/bin/bash
# One GPU call: decode phase times of the working tree and of ab/ builds,
# alternating, at 512 x 4K, one 4K frame and 64 x 1080p (every run checks the
# decoded frames against the input).  Usage: bash tools/gpu_abdec.sh TAG DIR...
export TMPDIR=/tmp; TAG=$1; shift; O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do for d in - "$@"; do
  if [ "$d" = "-" ]; then lib=""; else lib="NICE_LIB_PATH=$d/libnice_hip.so"; fi
  for sh in "512 3" "1 5" "64 3 1920 1080"; do echo "== [$d] $sh"; env $lib timeout -k 10 200 python tools/phase_time.py $sh 2>&1 | grep -E "decode|Error|assert" || exit 1; done
done; done > $O/ab.log
cat $O/ab.log
