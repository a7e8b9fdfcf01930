#!/bin/bash
# DRAM-side byte counters (tools/pmc_dram.txt) for the stencil kernels at N=512 fp64, plus the
# calibration kernel with a known byte count and the same access width / store policy
# (copy_width's read2write2<double, nt>: 8 B per lane, 4 GiB read + 4 GiB written per dispatch).
# Each step under its own limit; stops at the first failure.
cd "$(dirname "$0")/.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
A="512 1 pi pi pi 1 100 --format none --quiet"
set -e
timeout -k 10 400 tools/pmc_passes.sh cal tools/pmc_dram.txt "read2write2<double, true>" -- tools/microbench/copy_width
timeout -k 10 150 tools/pmc_passes.sh tb2 tools/pmc_dram.txt "k_tb2<double, false" -- $W $A --kernel tb2
timeout -k 10 150 tools/pmc_passes.sh march4nt tools/pmc_dram.txt "k_march<double, false" -- $W $A --kernel march4nt
timeout -k 10 150 tools/pmc_passes.sh tb3 tools/pmc_dram.txt "k_tb3<double, false" -- $W $A --kernel tb3
