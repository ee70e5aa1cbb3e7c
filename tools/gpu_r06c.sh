# SQ counters of the classify kernels: slide (default) and pair (NICE_ENC_NO_SLIDE=1), 32 frames
export TMPDIR=/tmp
bash tools/pmc_kernel.sh r06c_slide 32 "classify" > gpurun_out/r06c_slide.txt 2>&1 || exit 1
NICE_ENC_NO_SLIDE=1 bash tools/pmc_kernel.sh r06c_pair 32 "classify" > gpurun_out/r06c_pair.txt 2>&1 || exit 1
cat gpurun_out/r06c_slide.txt gpurun_out/r06c_pair.txt
