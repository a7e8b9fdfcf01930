#!/bin/bash
# round 4: kernel trace of the 8-rank 2x2x2 overlap-on run (N=1024 K=20 tb4 fma, zero-cost
# loopback): when do the shells and the interiors run relative to each other
mkdir -p gpurun_out
export TMPDIR=/tmp
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_ov -o ov -- $B 1024 8 pi pi pi 1 20 --ranks 8 --dims 2,2,2 \
  --math fma --overlap on --repeat 1 --warmup 1 --json --quiet --format none > gpurun_out/trace_ov.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_off -o off -- $B 1024 8 pi pi pi 1 20 --ranks 8 --dims 2,2,2 \
  --math fma --overlap off --graph off --repeat 1 --warmup 1 --json --quiet --format none > gpurun_out/trace_off.log 2>&1 || exit 1
tail -2 gpurun_out/trace_ov.log gpurun_out/trace_off.log
