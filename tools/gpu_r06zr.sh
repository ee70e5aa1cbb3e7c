#!/bin/bash
# r06zr: dec_place SMALL_DIFF constant by arithmetic (ab/sdlar) vs the table
# (working tree), 512 4K frames, then the full profile of the tree.
set -e
O=gpurun_out/r06zr; mkdir -p $O
for rep in 1 2; do
  for d in - ab/sdlar; do
    if [ "$d" = "-" ]; then unset NICE_LIB_PATH; else export NICE_LIB_PATH=$d/libnice_hip.so; fi
    echo "== [$d]"
    timeout -k 10 200 python tools/phase_time.py 512 3 2>&1 | grep -E "decode F|rror"
  done
done > $O/ab_sdl.log 2>&1
unset NICE_LIB_PATH
cat $O/ab_sdl.log
bash tools/gpu_profile.sh r06zr
timeout -k 10 300 bash tools/pmc_kernel.sh r06zr_sq 32 "nice::" > $O/pmc_sq.txt 2>&1
