#!/bin/bash
# round 4: fused fp64 fma leapfrog (stencil_math leap_fm) + predicated ring / per-tile LDS objects in
# k_tbn: parity tests, A/B (nofuse, nopred, onelds), then the overlap CU-reserve study and PMC
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_tb_kernels.py -m gpu -x -q -k "fma or tb4 or tbn or fp32 or delta or auto" --timeout 300 --timeout-method thread > gpurun_out/gputest_fused.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gputest_fused.log; [ $rc -eq 0 ] || exit $rc
tools/r4_ab_multi.sh 2 main:tb4:0 g1:tb4:0 g2:tb4:0 nofuse:tb4:0 nopred:tb4:0 onelds:tb4:0 main:tb3:0 nofuse:tb3:0 || exit 1
EXTRA="--math exact" tools/r4_ab_multi.sh 1 main:tb4:0 g1:tb4:0 g2:tb4:0 nopred:tb4:0 onelds:tb4:0 || exit 1
timeout -k 10 700 tools/archive/r4_batch7.sh > gpurun_out/overlap_cus.log 2>&1; rc=$?; cat gpurun_out/overlap_cus.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 480 tools/archive/r4_pmc2.sh > gpurun_out/pmc_r4b.log 2>&1; rc=$?; cat gpurun_out/pmc_r4b.log; exit $rc
