#!/bin/bash
# Work-item length (planes per marching work item) sweep of the default fp64 fma kernel, N=512.
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
for rep in 1 2; do
  for c in 0 64 128 171 256 512; do
    echo -n "rep=$rep chunk=$c: "
    timeout -k 10 120 $B ${N:-512} 1 pi pi pi 1 100 --math fma --chunk $c --repeat 5 --warmup 1 --json --quiet --format none \
      | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'])" || exit 1
  done
done
