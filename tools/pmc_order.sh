#!/bin/bash
cd "$(dirname "$0")/.."
export WAVE3D_TILE_ORDER=j
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
timeout -k 10 150 tools/pmc_passes.sh w8j tools/pmc_dram.txt k_tb2 -- $W 512 1 pi pi pi 1 100 --kernel tb2r2w8 --format none --quiet &&
timeout -k 10 150 tools/pmc_passes.sh w16k2j tools/pmc_dram.txt k_tb2 -- $W 512 1 pi pi pi 1 100 --kernel tb2r2w16k2 --format none --quiet
