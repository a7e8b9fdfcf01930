#!/bin/bash
# Cost of the per-sweep phase timers on the multi-rank path: 8 simulated ranks (2x2x2, loopback
# halos) at N=1024 fp64 K=100 on one GPU, timers on vs WAVE3D_NO_TIMERS=1, with direct launches
# (timing events) and with the hipGraph (stamp kernels). Arms alternated, best of 3 solves.
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
N=${N:-1024}
for rep in 1 2; do
  for g in off auto; do
    for nt in 0 1; do
      echo -n "graph=$g no_timers=$nt "
      WAVE3D_NO_TIMERS=$nt timeout -k 10 120 $B $N 1 pi pi pi 1 100 --ranks 8 --dims 2,2,2 --graph $g \
          --overlap ${OV:-off} --repeat 3 --warmup 1 --json --quiet --format none \
        | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), r['graph'], round(r['exchange_ms'],2), round(r['comm_ms'],2))" || exit 1
    done
  done
done
