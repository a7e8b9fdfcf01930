#!/bin/bash
# Tile-shape / XCD-order A/B of the temporal-blocking sweep (N=512 fp64 K=100), alternating
# arms each round so drift hits all of them; then the memory-side byte counters per arm.
cd "$(dirname "$0")/.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
A="512 1 pi pi pi 1 100 --format none --quiet --json --repeat 5 --warmup 1"
for rep in 1 2 3; do
  for arm in "tb2" "tb2r2w8" "tb2r2w16" "tb2 X" "tb2r2w8 X"; do
    k=${arm% X}; x=0; [ "$arm" != "$k" ] && x=1
    echo -n "arm=$k xcd=$x "
    WAVE3D_XCD_SWIZZLE=$x timeout -k 10 90 $W $A --kernel $k || exit 1
  done
done
