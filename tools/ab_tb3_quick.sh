set -e
tools/ab_kernels.sh "tb2r2w8 tb3 tb3r1w8" 2 -- 512 1 pi pi pi 1 100 --warmup 1 --repeat 3 > gpurun_out/ab_tb3_spill_512.log
