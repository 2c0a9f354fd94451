K_EXPR="generator or genome or chunked" bash tools/gpu_gen.sh > gpurun_out/gen4.txt 2>&1 && bash tools/pmc_sq.sh > gpurun_out/pmc4.txt 2>&1
