set -e
export NICE_PT_ENC_ONLY=1
for rep in 1 2; do for d in - ab/hprobe; do
  if [ "$d" = "-" ]; then unset NICE_LIB_PATH; else export NICE_LIB_PATH=$d/libnice_hip.so; fi
  echo "== [$d]"; timeout -k 10 200 python tools/phase_time.py 512 3 2>&1 | grep -E "encode F|rror" | cut -c1-140
done; done
