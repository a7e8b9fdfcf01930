#!/bin/bash
# config 5's grid and scheme on one GPU: N=2048 fp32 increment form K=200 --math fma, tb3 vs tb4
cd "$(dirname "$0")/../.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
for rep in 1 2; do
  for k in tb3 tb4 auto; do
    echo -n "rep=$rep kernel=$k "
    timeout -k 10 300 $W 2048 1 pi pi pi 1 200 --dtype fp32 --scheme delta --math fma --kernel $k --repeat 2 --warmup 1 \
        --json --quiet --format none | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.6g' % r['linf_abs'], r['kernel'])" || exit 1
  done
done
