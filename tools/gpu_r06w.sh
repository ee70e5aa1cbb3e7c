#!/bin/bash
# round 6: encoder GPU tests, then encode A/B at 512 x 4K and one 4K frame
export TMPDIR=/tmp; TAG=$1; shift; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_pack_cap.py tests/test_long_codes.py tests/test_gpu_parity.py \
  tests/test_slide.py tests/test_sharded.py tests/test_golden.py tests/test_tables.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for d in - "$@"; do
  if [ "$d" = "-" ]; then lib=""; else lib="NICE_LIB_PATH=$d/libnice_hip.so"; fi
  for sh in "512 3" "1 5"; do echo "== [$d] $sh"; env $lib timeout -k 10 200 python tools/phase_time.py $sh 2>&1 | grep -E "encode|Error|assert" || exit 1; done
done; done > $O/ab.log
cat $O/ab.log
