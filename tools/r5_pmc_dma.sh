#!/bin/bash
# Round 5: PMC passes (tools/pmc_l2.txt) of the LDS-DMA k_tbn<double,4> fma sweep vs the round-4
# register-staged build (gpurun_ab/old), N=512 K=40; plus the box's counter list.
set -e
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
run() { tag=$1; bin=$2; shift 2; tools/pmc_passes.sh "$tag" ${PMCFILE:-tools/pmc_l2.txt} "k_tbn<double, 4, false" -- $bin 512 1 pi pi pi 1 40 --math fma --quiet --format none --graph off "$@" > /dev/null; echo "== $tag"; cat gpurun_out/$tag/summary.txt; }
run ${TAG:-pmc_r5_dma} $B ${PMCEXTRA:-}
run ${TAG:-pmc_r5}_old gpurun_ab/old/wave3d ${PMCEXTRA:-}

