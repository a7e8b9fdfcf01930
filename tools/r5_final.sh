#!/bin/bash
# Round 5 evidence for the shipped sweep: bench.py (headline config), rocprofv3 kernel stats of a
# bench-shaped run, and PMC passes of the fp64 fma k_tbn<4> against the round-4 build.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench_r5.json 2> gpurun_out/bench_r5.err || exit $?
tail -1 gpurun_out/bench_r5.json
timeout -k 10 300 python bench.py >> gpurun_out/bench_r5.json 2>> gpurun_out/bench_r5.err || exit $?
tail -1 gpurun_out/bench_r5.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5 -o run -- \
    3d-wave-equation-mpi-cuda_amd/build/wave3d 512 1 pi pi pi 1 100 --math fma --repeat 3 --quiet --format none \
    > gpurun_out/prof_r5.log 2>&1 || exit $?
find gpurun_out/prof_r5 -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats_r5.csv \;
PMCFILE=tools/pmc_l2.txt TAG=pmc_r5_final tools/r5_pmc_dma.sh > gpurun_out/pmc_r5_final.txt 2>&1 || exit $?
PMCFILE=tools/pmc_sq_r5.txt TAG=pmc_r5_finalsq tools/r5_pmc_dma.sh > gpurun_out/pmc_r5_finalsq.txt 2>&1 || exit $?
echo done
