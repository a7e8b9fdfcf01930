#!/bin/bash
# Increment form on tb3: bitwise tests vs the OpenMP oracle, then tb2 vs tb3 tiles (fp32 delta).
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_solver.py -k "delta or tb3" -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/tb3delta_tests.log 2>&1
tail -2 gpurun_out/tb3delta_tests.log
tools/ab_kernels.sh "tb2r2w8 tb2 tb3 tb3r1w8" 2 -- 512 1 pi pi pi 1 100 --dtype fp32 --scheme delta --warmup 1 --repeat 3 > gpurun_out/ab_delta_512.log
tools/ab_kernels.sh "tb2 tb3 tb3r1w8" 1 -- 2048 1 pi pi pi 1 200 --dtype fp32 --scheme delta --warmup 1 --repeat 2 > gpurun_out/ab_delta_2048.log
