#!/bin/bash
# round 4: final tb4 configuration (ring branches, per-tile LDS objects, fused fp64 fma leapfrog):
# GPU suite, bench.py fma / exact, A/B of the LDS gather variants, PMC of the shipped sweep
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4d.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gputest_r4d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r4d.json 2> gpurun_out/bench_r4d.err || exit 1
cat gpurun_out/bench_r4d.json
timeout -k 10 300 python bench.py --math exact > gpurun_out/bench_r4d_exact.json 2> gpurun_out/bench_r4d_exact.err || exit 1
cat gpurun_out/bench_r4d_exact.json
tools/r4_ab_multi.sh 2 main:tb4:0 g1np:tb4:0 g2np:tb4:0 || exit 1
EXTRA="--math exact" tools/r4_ab_multi.sh 1 main:tb4:0 g1np:tb4:0 g2np:tb4:0 || exit 1
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
timeout -k 10 300 tools/pmc_passes.sh pmc_r4_tb4final tools/pmc_l2.txt "k_tbn<double, 4, false" -- $B 512 1 pi pi pi 1 40 --math fma --quiet --format none --graph off > /dev/null || exit 1
cat gpurun_out/pmc_r4_tb4final/summary.txt
