#!/bin/bash
# Round-4 PMC passes (tools/pmc_l2.txt) of the shipped sweeps after the tb4 switch:
#   pmc_r4_tb4m      k_tbn<double, 4> fma, N=512 K=40 (bench.py's kernel, masks as products, no SLP)
#   pmc_r4_tb4x      k_tbn<double, 4> exact, N=512 K=40
#   pmc_r4_f32d_sc   k_tb3<float> increment form, exact, N=1024 K=40: the shipped (scalar) build
#   pmc_r4_f32d_pk   the same with LLVM's SLP pairing (v_pk_* fp32; gpurun_ab/slp, the round-3 build mode)
set -e
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
S=gpurun_ab/slp/wave3d
run() { tag=$1; match=$2; shift 2; tools/pmc_passes.sh "$tag" tools/pmc_l2.txt "$match" -- "$@" > /dev/null; echo "== $tag"; cat gpurun_out/$tag/summary.txt; }
run pmc_r4_tb4m "k_tbn<double, 4, false" $B 512 1 pi pi pi 1 40 --math fma --quiet --format none --graph off
run pmc_r4_tb4x "k_tbn<double, 4, false" $B 512 1 pi pi pi 1 40 --math exact --quiet --format none --graph off
run pmc_r4_f32d_sc "k_tb3<float, false, 2, 8, true" $B 1024 1 pi pi pi 1 40 --dtype fp32 --scheme delta --math exact --quiet --format none --graph off
run pmc_r4_f32d_pk "k_tb3<float, false, 2, 8, true" $S 1024 1 pi pi pi 1 40 --dtype fp32 --scheme delta --math exact --quiet --format none --graph off
