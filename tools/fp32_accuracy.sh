#!/bin/bash
# fp32 accuracy floor: leapfrog vs increment form (--scheme delta) against fp64, one GPU.
cd "$(dirname "$0")/.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
run() { echo -n "$* "; timeout -k 10 300 $W "$@" --json --format none --quiet || exit 1; }
run 1024 1 pi pi pi 1 100 --repeat 2
run 1024 1 pi pi pi 1 100 --dtype fp32 --repeat 2
run 1024 1 pi pi pi 1 100 --dtype fp32 --scheme delta --repeat 2
run 2048 1 pi pi pi 1 200 --dtype fp32 --repeat 2
run 2048 1 pi pi pi 1 200 --dtype fp32 --scheme delta --repeat 2
run 2048 1 pi pi pi 1 200 --kernel march2 --repeat 1
