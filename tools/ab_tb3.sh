#!/bin/bash
# tb3 register/instruction-diet check: isolated + solver tb3 tests, then tb2 vs tb3 tiles.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tb_kernels.py tests/test_gpu_solver.py -k tb3 -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/tb3_tests.log 2>&1
tail -3 gpurun_out/tb3_tests.log
tools/ab_kernels.sh "tb2r2w8 tb3 tb3r1w16 tb3r1w8" 2 -- 512 1 pi pi pi 1 100 --warmup 1 --repeat 3 > gpurun_out/ab_tb3_fp64_512.log
tools/ab_kernels.sh "tb2r2w8 tb3 tb3r1w8" 2 -- 512 1 pi pi pi 1 100 --warmup 1 --repeat 3 --dtype fp32 > gpurun_out/ab_tb3_fp32_512.log
tools/ab_kernels.sh "tb2r2w8 tb3 tb3r1w8" 1 -- 1024 1 pi pi pi 1 100 --warmup 1 --repeat 2 > gpurun_out/ab_tb3_fp64_1024.log
tools/ab_kernels.sh "tb2r2w8 tb3 tb3r1w8" 1 -- 2048 1 pi pi pi 1 200 --warmup 1 --repeat 2 --dtype fp32 > gpurun_out/ab_tb3_fp32_2048.log
