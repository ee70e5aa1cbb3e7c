#!/bin/bash
# round 6: decode GPU tests, then decode A/B at 512 x 4K, one 4K frame, 64 x 1080p, one 1080p frame, 4 x 4K
export TMPDIR=/tmp; TAG=$1; shift; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "decode or sync or settle or fuzz or parity or async or crafted or flow or strict or roundtrip or slice" > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for d in - "$@"; do
  if [ "$d" = "-" ]; then lib=""; else lib="NICE_LIB_PATH=$d/libnice_hip.so"; fi
  for sh in "512 3" "1 5" "64 3 1920 1080" "1 5 1920 1080" "4 5"; do echo "== [$d] $sh"; env $lib timeout -k 10 200 python tools/phase_time.py $sh 2>&1 | grep -E "decode|Error|assert" || exit 1; done
done; done > $O/ab.log
cat $O/ab.log
