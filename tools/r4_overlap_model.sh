#!/bin/bash
# Overlap with a modelled xGMI link on one GPU (round 4): P simulated ranks
# (default 8 as 2x2x2), N=1024 fp64 K=100 --math fma, loopback halos; --model-link G[,L] makes
# every exchange also wait the time its busiest peer link needs at G GB/s (+ L us) on one CU of
# the exchange stream. Arms: zero-cost exchange (no model) with overlap off / on; 50 GB/s + 5 us
# with overlap off / on. Best of 2 solves (after 1 warm-up), alternating rounds.
#   P=2 DIMS=2,1,1 KER=tb4 XARGS="--chunk 128" tools/r4_overlap_model.sh 2
cd "$(dirname "$0")/.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
rounds=${1:-2}; K=${K:-100}; N=${N:-1024}; KER=${KER:-tb3}; P=${P:-8}; DIMS=${DIMS:-2,2,2}
for rep in $(seq "$rounds"); do
  for arm in "off:" "on:" "off:--model-link 50,5" "on:--model-link 50,5"; do
    ov=${arm%%:*}; extra=${arm#*:}
    echo -n "round=$rep P=$P dims=$DIMS kernel=$KER ${XARGS:-} overlap=$ov ${extra:-zero-cost} "
    timeout -k 10 200 $W $N $P pi pi pi 1 $K --ranks $P --dims $DIMS --math fma --kernel $KER --overlap $ov $extra \
        ${XARGS:-} --repeat 2 --warmup 1 --json --quiet --format none \
      | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.6g' % r['linf_abs'], 'exch_ms', round(r.get('exchange_ms',0),1), 'loop_ms', round(r.get('loop_ms',0),1))" || exit 1
  done
done
