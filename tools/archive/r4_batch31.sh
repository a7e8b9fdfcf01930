#!/bin/bash
# round 4: k_tbn per element type (fp32: one LDS array + wave priority during the prefetch; fp64
# unchanged) vs the previous build (old): tb4 tests, then A/B fp32 fma / exact / increment form, fp64
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_tb_kernels.py tests/test_gpu_halo_selftest.py -m gpu -x -q -k "tb4 or tbn or fp32 or golden or delta" --timeout 300 --timeout-method thread > gpurun_out/gputest_tbn32.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest_tbn32.log; [ $rc -eq 0 ] || exit $rc
EXTRA="--dtype fp32" tools/r4_ab_multi.sh 2 main:tb4:0 old:tb4:0 || exit 1
EXTRA="--dtype fp32 --math exact" tools/r4_ab_multi.sh 2 main:tb4:0 old:tb4:0 || exit 1
EXTRA="--dtype fp32 --scheme delta --math exact" tools/r4_ab_multi.sh 1 main:tb4:0 old:tb4:0 || exit 1
tools/r4_ab_multi.sh 2 main:tb4:0 old:tb4:0 || exit 1
