#!/bin/bash
# Single-step kernel (march2) overlap: simulated 2x2x2 at N=1024 and one rank with RCCL self-send.
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
for o in "" "--no-overlap"; do
  echo -n "sim222 march2 ov=${o:-on} "; timeout -k 10 120 $B 1024 8 pi pi pi 1 100 --ranks 8 --dims 2,2,2 --kernel march2 $o --repeat 3 --warmup 1 --json --format none --quiet || exit 1
  echo -n "self march2 ov=${o:-on} "; timeout -k 10 120 python3 tools/dist_solve.py --backend hip --transport rccl -- 512 1 pi pi pi 1 100 --kernel march2 --x-self-transport $o --repeat 3 --warmup 1 | grep RESULT || exit 1
done
