#!/bin/bash
# Simulated 8 ranks on one GPU (N=1024, tb2): overlap on/off with the default 4 HIP hardware
# queues per process vs 16. Each simulated rank has a compute and a comm stream (16 streams):
# with 4 queues they are multiplexed and a rank's shells queue behind other ranks' interiors.
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
for rep in 1 2; do for q in 4 16; do for d in 2,2,2 8,1,1; do for o in "" "--no-overlap"; do
  echo -n "queues=$q dims=$d ov=${o:-on} "
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 $B 1024 8 pi pi pi 1 100 --ranks 8 --dims $d $o --repeat 3 --warmup 1 --json --format none --quiet || exit 1
done; done; done; done
