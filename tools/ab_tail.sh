#!/bin/bash
# Tail-aware work-item length (chunk_for_slots) vs the previous build: simulated 8-rank N=1024
# (2x2x2 / 8x1x1, overlap on and off) and the single-rank grids; plus the tb2 tests.
set -e
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest tests/test_gpu_tb_kernels.py tests/test_gpu_solver.py -k "tb2 or overlap or auto or delta" -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/tail_tests.log 2>&1
tail -2 gpurun_out/tail_tests.log
tools/ab_bins.sh 2 -- 1024 8 pi pi pi 1 100 --ranks 8 --dims 2,2,2 --warmup 1 --repeat 2 > gpurun_out/abtail_222_on.log
tools/ab_bins.sh 2 -- 1024 8 pi pi pi 1 100 --ranks 8 --dims 2,2,2 --no-overlap --warmup 1 --repeat 2 > gpurun_out/abtail_222_off.log
tools/ab_bins.sh 2 -- 1024 8 pi pi pi 1 100 --ranks 8 --dims 8,1,1 --warmup 1 --repeat 2 > gpurun_out/abtail_811_on.log
tools/ab_bins.sh 2 -- 512 1 pi pi pi 1 100 --warmup 1 --repeat 3 > gpurun_out/abtail_512.log
