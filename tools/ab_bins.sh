#!/bin/bash
# A/B of two builds (gpurun_ab/old/wave3d vs the tree's build/wave3d), alternating:
#   tools/ab_bins.sh REPS -- <wave3d args...>
cd "$(dirname "$0")/.."
reps=$1; shift
[ "$1" = "--" ] && shift
for rep in $(seq "$reps"); do
  for v in old new; do
    if [ $v = old ]; then B=gpurun_ab/old/wave3d; else B=3d-wave-equation-mpi-cuda_amd/build/wave3d; fi
    echo -n "$v "
    timeout -k 10 120 $B "$@" --json --format none --quiet || exit 1
  done
done
