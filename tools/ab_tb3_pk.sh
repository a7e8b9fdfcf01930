#!/bin/bash
# Packed-fp32 tb3 (L = 2) vs the scalar instantiation (WAVE3D_TB3_PK=0): tb3 tests, then A/B.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tb_kernels.py tests/test_gpu_solver.py -k "tb3 or fp32" -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/tb3pk_tests.log 2>&1
tail -2 gpurun_out/tb3pk_tests.log
tools/ab_env.sh WAVE3D_TB3_PK "1 0" 3 -- 512 1 pi pi pi 1 100 --dtype fp32 --warmup 1 --repeat 3 > gpurun_out/ab_tb3pk_512.log
tools/ab_env.sh WAVE3D_TB3_PK "1 0" 2 -- 2048 1 pi pi pi 1 200 --dtype fp32 --warmup 1 --repeat 2 > gpurun_out/ab_tb3pk_2048.log
