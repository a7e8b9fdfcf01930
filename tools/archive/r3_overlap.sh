#!/bin/bash
# Overlap on/off of the default fp64 fma kernel on simulated ranks (one GPU, loopback halos).
# Best of 3 solves.
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
run() {
  timeout -k 10 200 $B "$@" --math fma --repeat 3 --warmup 1 --json --quiet --format none \
    | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'], 'overlap', r['overlap'], 'exch_ms', round(r['exchange_ms'],1))"
}
for rep in 1 2; do
  for ov in off on; do
    echo -n "rep=$rep N=1024 ranks=8 2x2x2 overlap=$ov: "; run 1024 1 pi pi pi 1 100 --ranks 8 --dims 2,2,2 --overlap $ov || exit 1
    echo -n "rep=$rep N=1024 ranks=4 2x2x1 overlap=$ov: "; run 1024 1 pi pi pi 1 100 --ranks 4 --dims 2,2,1 --overlap $ov || exit 1
  done
  echo -n "rep=$rep N=512 1 rank (fused wrap, graph): "; run 512 1 pi pi pi 1 100 || exit 1
done
