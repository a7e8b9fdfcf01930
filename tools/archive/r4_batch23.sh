#!/bin/bash
# round 4: PMC of the max-ilp build's sweeps (tb4 fp64 fma / exact, tb3 fp32 increment form) and
# every BASELINE config on that build
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
run() { tag=$1; match=$2; shift 2; tools/pmc_passes.sh "$tag" tools/pmc_l2.txt "$match" -- "$@" > /dev/null; echo "== $tag"; cat gpurun_out/$tag/summary.txt; }
run pmc_r4_ilp_tb4m "k_tbn<double, 4, false" $B 512 1 pi pi pi 1 40 --math fma --quiet --format none --graph off
run pmc_r4_ilp_tb4x "k_tbn<double, 4, false" $B 512 1 pi pi pi 1 40 --math exact --quiet --format none --graph off
run pmc_r4_ilp_f32d "k_tb3<float, false, 2, 8, true" $B 1024 1 pi pi pi 1 40 --dtype fp32 --scheme delta --math exact --quiet --format none --graph off
tools/archive/r4_configs.sh
