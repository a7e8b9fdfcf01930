#!/bin/bash
# A/B over an environment switch of one binary, alternating values so drift hits all arms:
#   tools/ab_env.sh VAR "v1 v2 ..." REPS -- <wave3d args...>
# prints "VAR=v <json>" per run; stops at the first failing run.
cd "$(dirname "$0")/.."
var=$1; vals=$2; reps=$3; shift 3
[ "$1" = "--" ] && shift
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
for rep in $(seq "$reps"); do
  for v in $vals; do
    echo -n "$var=$v "
    env "$var=$v" timeout -k 10 90 $B "$@" --json --format none --quiet || exit 1
  done
done
