#!/bin/bash
# 64- vs 128-column tb2 tiles (N=512 fp64 K=100), alternating; then memory-side bytes.
cd "$(dirname "$0")/.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
A="512 1 pi pi pi 1 100 --format none --quiet --json --repeat 5 --warmup 1"
for rep in 1 2 3; do
  for k in tb2r2w8 tb2r2w8k2 tb2r2w8k2o4 tb2r2w16k2; do
    echo -n "arm=$k "; timeout -k 10 90 $W $A --kernel $k || exit 1
  done
done
