#!/bin/bash
# --halo direct (one round) vs rounds (x, y, z) on simulated ranks (one GPU, loopback D2D halos,
# hipGraph), the fp64 default kernel, N=1024 8 ranks 2x2x2 and 4 ranks 2x2x1, overlap on/off.
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
for rep in 1 2; do
for cfg in "1024 8 2,2,2" "1024 4 2,2,1"; do
  set -- $cfg
  for h in direct rounds; do
    for ov in off on; do
      echo -n "N=$1 ranks=$2 dims=$3 halo=$h overlap=$ov: "
      timeout -k 10 200 $B $1 1 pi pi pi 1 100 --ranks $2 --dims $3 --math fma --halo $h --overlap $ov \
          --repeat 3 --warmup 1 --json --quiet --format none \
        | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'], round(r['exchange_ms'],1), round(r['comm_ms'],1))" || exit 1
    done
  done
done
done
