#!/bin/bash
cd "$(dirname "$0")/.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
for rep in 1 2; do for s in leapfrog delta; do for k in tb2r4 tb2r2w8 tb2; do
  echo -n "N=512 scheme=$s kernel=$k "
  timeout -k 10 100 $W 512 1 pi pi pi 1 100 --dtype fp32 --scheme $s --kernel $k --repeat 5 --warmup 1 --json --format none --quiet || exit 1
done; done; done
for k in tb2r2w8 tb2; do echo -n "N=512 fp64 delta kernel=$k "; timeout -k 10 100 $W 512 1 pi pi pi 1 100 --scheme delta --kernel $k --repeat 5 --warmup 1 --json --format none --quiet || exit 1; done
