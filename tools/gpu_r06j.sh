export TMPDIR=/tmp; O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_flow.py tests/test_split.py tests/test_width_sweep.py tests/test_rows_wrap.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for e in "NICE_DEC_SPLIT=2" "NICE_X=0"; do echo "== $e 16x8K"; env $e timeout -k 10 200 python tools/phase_time.py 16 3 7680 4320 2>&1 | grep decode || exit 1; done > $O/ab.log
for e in "NICE_DEC_SPLIT=2" "NICE_X=0"; do echo "== $e 1x8K"; env $e timeout -k 10 200 python tools/phase_time.py 1 3 7680 4320 2>&1 | grep decode || exit 1; done >> $O/ab.log
for e in "NICE_DEC_FLOW=0" "NICE_X=0"; do echo "== $e 64x8K"; env $e timeout -k 10 200 python tools/phase_time.py 64 3 7680 4320 2>&1 | grep decode || exit 1; done >> $O/ab.log
echo "== 16384^2"; timeout -k 10 200 python tools/phase_time.py 1 2 16384 16384 2>&1 | grep decode >> $O/ab.log || exit 1
cat $O/ab.log
