#!/bin/bash
# First-solve cost of the CLI (what one `wave3d N 1 ...` run reports) vs warm solves.
set -e
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
for r in 1 2 3; do
    echo -n "cold "; timeout -k 10 90 $B 512 1 pi pi pi 1 100 --json --format none --quiet
    echo -n "warm "; timeout -k 10 90 $B 512 1 pi pi pi 1 100 --warmup 1 --repeat 3 --json --format none --quiet
done
