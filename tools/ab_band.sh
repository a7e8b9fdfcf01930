#!/bin/bash
# Tile order A/B: j-fastest (default) vs XCD bands, tb2 tiles at N=512 and N=1024, then the
# memory-side bytes of the band order (tools/pmc_dram.txt).
cd "$(dirname "$0")/.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
for rep in 1 2 3; do
  for n in 512 1024; do for k in tb2r2w8 tb2r2w16; do for o in j band; do
    echo -n "N=$n arm=$k order=$o "
    WAVE3D_TILE_ORDER=$o timeout -k 10 90 $W $n 1 pi pi pi 1 100 --format none --quiet --json --repeat 5 --warmup 1 --kernel $k || exit 1
  done; done; done
done
export WAVE3D_TILE_ORDER=band
timeout -k 10 150 tools/pmc_passes.sh w8band tools/pmc_dram.txt k_tb2 -- $W 512 1 pi pi pi 1 100 --kernel tb2r2w8 --format none --quiet
