#!/bin/bash
# XCD placement A/B: band order (default) vs contiguous-range swizzle + k-fastest decode (every
# XCD a compact 2-D patch of tiles, balanced for any tile count), 1 GPU N=512 and the simulated
# 2x2x2 overlap run (interior tiles_j = 30: the band order falls back to j there).
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
A="--format none --quiet --json --repeat 5 --warmup 1"
for rep in 1 2 3; do
  echo -n "n512 band ";      timeout -k 10 90 $B 512 1 pi pi pi 1 100 $A || exit 1
  echo -n "n512 swz-k ";     WAVE3D_XCD_SWIZZLE=1 WAVE3D_TILE_ORDER=k timeout -k 10 90 $B 512 1 pi pi pi 1 100 $A || exit 1
  echo -n "sim222 band ";    timeout -k 10 120 $B 1024 8 pi pi pi 1 100 --ranks 8 --dims 2,2,2 --repeat 3 --warmup 1 --json --format none --quiet || exit 1
  echo -n "sim222 swz-k ";   WAVE3D_XCD_SWIZZLE=1 WAVE3D_TILE_ORDER=k timeout -k 10 120 $B 1024 8 pi pi pi 1 100 --ranks 8 --dims 2,2,2 --repeat 3 --warmup 1 --json --format none --quiet || exit 1
  echo -n "sim222off band "; timeout -k 10 120 $B 1024 8 pi pi pi 1 100 --ranks 8 --dims 2,2,2 --no-overlap --repeat 3 --warmup 1 --json --format none --quiet || exit 1
  echo -n "sim222off swz-k "; WAVE3D_XCD_SWIZZLE=1 WAVE3D_TILE_ORDER=k timeout -k 10 120 $B 1024 8 pi pi pi 1 100 --ranks 8 --dims 2,2,2 --no-overlap --repeat 3 --warmup 1 --json --format none --quiet || exit 1
done
