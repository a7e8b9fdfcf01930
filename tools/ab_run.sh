#!/bin/bash
# A/B: old (division) vs new (exact argmax) binaries, alternating
cd "$(dirname "$0")/.."
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then B=gpurun_ab/wave3d; else B=3d-wave-equation-mpi-cuda_amd/build/wave3d; fi
    for k in tb2 march2; do
      echo -n "$v $k "
      timeout -k 10 60 $B 512 1 pi pi pi 1 100 --kernel $k --repeat 5 --warmup 1 --json --format none --quiet || exit 1
    done
  done
done
