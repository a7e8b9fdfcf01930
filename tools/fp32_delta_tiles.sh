#!/bin/bash
# fp32 N=2048 K=200: tile shapes for leapfrog and the increment form, alternating.
cd "$(dirname "$0")/.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
for rep in 1 2; do
  for s in leapfrog delta; do for k in tb2r4 tb2r2w8 tb2; do
    echo -n "scheme=$s kernel=$k "
    timeout -k 10 200 $W 2048 1 pi pi pi 1 200 --dtype fp32 --scheme $s --kernel $k --repeat 2 --json --format none --quiet || exit 1
  done; done
done
