#!/bin/bash
# tb2r2w8 (band order) work-item length sweep at N=512 / 1024: planes per work item vs rounds of
# workgroups (2 per CU resident) and the per-item 2-plane prologue.
cd "$(dirname "$0")/.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
for rep in 1 2; do
  for n in 512 1024; do for c in 0 64 128 171 256; do
    echo -n "N=$n chunk=$c "
    timeout -k 10 90 $W $n 1 pi pi pi 1 100 --format none --quiet --json --repeat 5 --warmup 1 --chunk $c || exit 1
  done; done
done
