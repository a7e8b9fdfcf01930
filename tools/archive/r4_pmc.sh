#!/bin/bash
# Round-4 PMC passes (tools/pmc_l2.txt: wave states, instruction mix, LDS conflicts, L2 hit / miss,
# memory-side requests and bytes) of the deep sweeps, N=512 fp64 K=40 --math fma (non-first sweeps),
# and of the fp32 increment-form tb3 sweep (config 5's kernel) at N=1024 K=40.
set -e
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
run() { tag=$1; match=$2; shift 2; tools/pmc_passes.sh "$tag" tools/pmc_l2.txt "$match" -- "$@" > /dev/null; echo "== $tag"; cat gpurun_out/$tag/summary.txt; }
run pmc_r4_tb3 "k_tb3<double, false, 2, 8" $B 512 1 pi pi pi 1 40 --math fma --kernel tb3 --quiet --format none --graph off
run pmc_r4_tbn3 "k_tbn<double, 3, false" $B 512 1 pi pi pi 1 40 --math fma --kernel tbn3 --quiet --format none --graph off
run pmc_r4_tb4 "k_tbn<double, 4, false" $B 512 1 pi pi pi 1 40 --math fma --kernel tb4 --quiet --format none --graph off
run pmc_r4_tb3_fp32d "k_tb3<float, false, 2, 8, true" $B 1024 1 pi pi pi 1 40 --dtype fp32 --scheme delta --math fma --quiet --format none --graph off
