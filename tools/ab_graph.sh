#!/bin/bash
# hipGraph replay vs direct launches (the path every multi-process run takes: graph_eligible()
# excludes an external transport), tb2r2w8 fp64 N=512 and the 2x2x2 simulated N=1024.
set -e
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
run() { echo -n "$1 "; shift; timeout -k 10 120 $B "$@" --json --format none --quiet; }
for rep in 1 2 3; do
  run graph-on 512 1 pi pi pi 1 100 --graph on --warmup 1 --repeat 3
  run graph-off 512 1 pi pi pi 1 100 --graph off --warmup 1 --repeat 3
done > gpurun_out/ab_graph.log
