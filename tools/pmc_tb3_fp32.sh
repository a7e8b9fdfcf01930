#!/bin/bash
# PMC passes of the fp32 tb3 sweep (auto kernel for fp32, N=512 K=40), one rocprofv3 run per pass.
set -e
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
tools/pmc_passes.sh pmc_tb3_fp32 tools/pmc_tb.txt k_tb3 -- $B 512 1 pi pi pi 1 40 --dtype fp32 --quiet --format none
