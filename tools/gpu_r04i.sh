mkdir -p gpurun_out/r04i
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r04i/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r04i/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04i/pytest_gpu.log
bash tools/abn.sh 512 ab/s1 ab/s2 > gpurun_out/r04i/ab_sync.log 2>&1 || exit 1
bash tools/ab_env.sh 512 - NICE_DEC_SERIAL_PLACE=1 > gpurun_out/r04i/ab_place.log 2>&1 || exit 1
grep -E "==|decode" gpurun_out/r04i/ab_sync.log gpurun_out/r04i/ab_place.log
