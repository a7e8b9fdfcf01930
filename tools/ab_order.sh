#!/bin/bash
# Tile order A/B (k-fastest vs j-fastest block ids) for 64- and 128-column tb2 tiles.
cd "$(dirname "$0")/.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
A="512 1 pi pi pi 1 100 --format none --quiet --json --repeat 5 --warmup 1"
for rep in 1 2 3; do
  for k in tb2r2w8 tb2r2w16k2 tb2r2w8k2o4; do for o in k j; do
    echo -n "arm=$k order=$o "; WAVE3D_TILE_ORDER=$o timeout -k 10 90 $W $A --kernel $k || exit 1
  done; done
done
