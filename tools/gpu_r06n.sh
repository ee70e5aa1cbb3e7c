#!/bin/bash
# round 6: decode-side GPU tests, then the decode A/B (tools/gpu_abdec.sh) against ab builds
export TMPDIR=/tmp; TAG=$1; shift; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "decode or sync or settle or fuzz or parity or async or crafted or flow or strict or roundtrip" > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_abdec.sh $TAG "$@"
