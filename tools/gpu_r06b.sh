export TMPDIR=/tmp; O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_slide.py tests/test_classify_routes.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for e in "NICE_ENC_NO_SLIDE=1" "NICE_X=0" "NICE_ENC_NO_SLIDE=1" "NICE_X=0"; do echo "== $e"; env $e timeout -k 10 200 python tools/phase_time.py 512 3 2>&1 | grep encode; done > $O/ab.log
cat $O/ab.log
