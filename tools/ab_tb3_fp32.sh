set -e
tools/ab_kernels.sh "tb2r2w8 tb3 tb3r2w4" 3 -- 512 1 pi pi pi 1 100 --dtype fp32 > gpurun_out/ab_fp32_512.log
tools/ab_kernels.sh "tb2r2w8 tb3 tb3r2w4" 3 -- 512 1 pi pi pi 1 100 > gpurun_out/ab_fp64_512.log
tools/ab_kernels.sh "tb2r2w8 tb3" 2 -- 2048 1 pi pi pi 1 200 --dtype fp32 > gpurun_out/ab_fp32_2048.log
