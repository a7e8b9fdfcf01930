#!/bin/bash
# A/B over --kernel variants of one binary, alternating so drift hits all arms:
#   tools/ab_kernels.sh "k1 k2 ..." REPS -- <wave3d args without --kernel...>
# prints "<kernel> <json>" per run; stops at the first failing run.
cd "$(dirname "$0")/.."
ks=$1; reps=$2; shift 2
[ "$1" = "--" ] && shift
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
for rep in $(seq "$reps"); do
  for k in $ks; do
    echo -n "$k "
    timeout -k 10 90 $B "$@" --kernel "$k" --json --format none --quiet || exit 1
  done
done
