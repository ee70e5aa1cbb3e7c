bash tools/gpu_abenc.sh r06e 512 ab/slide_pin - || exit 1
bash tools/pmc_kernel.sh r06e_sq 32 "classify" > gpurun_out/r06e_sq.txt 2>&1 || exit 1
cat gpurun_out/r06e_sq.txt
