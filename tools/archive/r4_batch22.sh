#!/bin/bash
# round 4: more machine-scheduler strategies for the deep sweeps (hip_tbn + hip_tb3): itilp =
# iterative-ilp, itmin = iterative-minreg, ilptrk = max-ilp with the AMDGPU pressure trackers;
# main = the shipped max-ilp build
mkdir -p gpurun_out
tools/r4_ab_multi.sh 2 main:tb4:0 itilp:tb4:0 itmin:tb4:0 ilptrk:tb4:0 || exit 1
EXTRA="--dtype fp32" tools/r4_ab_multi.sh 1 main:tb4:0 itilp:tb4:0 itmin:tb4:0 ilptrk:tb4:0 || exit 1
EXTRA="--math exact --dtype fp32 --scheme delta" tools/r4_ab_multi.sh 1 main:tb3:0 itilp:tb3:0 itmin:tb3:0 ilptrk:tb3:0 || exit 1
