#!/bin/bash
# Ring-work balance across SIMDs (tb3): tb3 tests, then same-box A/B against the previous build.
set -e
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest tests/test_gpu_tb_kernels.py tests/test_gpu_solver.py -k "tb3 or delta" -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/tb3bal_tests.log 2>&1
tail -2 gpurun_out/tb3bal_tests.log
tools/ab_bins.sh 3 -- 512 1 pi pi pi 1 100 --kernel tb3r1w8 --warmup 1 --repeat 3 > gpurun_out/abbal_fp64_r1w8.log
tools/ab_bins.sh 2 -- 512 1 pi pi pi 1 100 --dtype fp32 --warmup 1 --repeat 3 > gpurun_out/abbal_fp32.log
tools/ab_kernels.sh "tb2r2w8 tb3r1w8" 2 -- 512 1 pi pi pi 1 100 --warmup 1 --repeat 3 > gpurun_out/abbal_vs_tb2.log
