#!/bin/bash
# Work-item length (planes per marching chunk) of the tb3 sweeps vs tb2r2w8, fp64 / fp32 N=512.
set -e
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
run() { echo -n "$1 "; shift; timeout -k 10 90 $B "$@" --json --format none --quiet; }
for rep in 1 2; do
  run "tb2r2w8-auto" 512 1 pi pi pi 1 100 --kernel tb2r2w8 --warmup 1 --repeat 3
  for c in 64 96 128 171 256; do
    run "tb3r1w8-c$c" 512 1 pi pi pi 1 100 --kernel tb3r1w8 --chunk $c --warmup 1 --repeat 3
  done
done > gpurun_out/chunk_tb3_fp64.log
for rep in 1 2; do
  for c in 64 96 128 171 256; do
    run "tb3-c$c" 512 1 pi pi pi 1 100 --dtype fp32 --chunk $c --warmup 1 --repeat 3
  done
done > gpurun_out/chunk_tb3_fp32.log
