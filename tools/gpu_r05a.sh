export TMPDIR=/tmp
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_strict_refill.py tests/test_width_sweep.py tests/test_sharded.py tests/test_pack_cap.py tests/test_split.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_new.log 2>&1; rc=$?; tail -15 $O/pytest_new.log; exit $rc
