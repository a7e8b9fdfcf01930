#!/bin/bash
# fp32 leapfrog vs increment form with the default (tb3) kernels, one MI355X, --math fma:
# L-inf abs of the final layer and Mpts/s (best of 3 solves). -> profiles/fp32_scheme_r4.txt
cd "$(dirname "$0")/.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
for cfg in "512 100" "2048 200"; do
  set -- $cfg
  for sch in leapfrog delta; do
    echo -n "N=$1 K=$2 fp32 $sch "
    timeout -k 10 300 $W $1 1 pi pi pi 1 $2 --dtype fp32 --scheme $sch --math fma --repeat 3 --warmup 1 \
        --json --quiet --format none \
      | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.6g' % r['linf_abs'], r['kernel'])" || exit 1
  done
  echo -n "N=$1 K=$2 fp64 leapfrog "
  timeout -k 10 300 $W $1 1 pi pi pi 1 $2 --math fma --repeat 2 --warmup 1 --json --quiet --format none \
    | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.6g' % r['linf_abs'], r['kernel'])" || exit 1
done
