export TMPDIR=/tmp; O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for d in ab/head8 -; do
  if [ "$d" = "-" ]; then lib=""; else lib="NICE_LIB_PATH=$d/libnice_hip.so"; fi
  for sh in "512 3" "1 5" "64 3 1920 1080"; do echo "== [$d] $sh"; env $lib timeout -k 10 200 python tools/phase_time.py $sh 2>&1 | grep decode || exit 1; done
done; done > $O/ab.log
cat $O/ab.log
