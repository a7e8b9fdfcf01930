#!/bin/bash
# round 4: k_tbn's rejected switches re-tried under max-ilp (pred = W3D_TBN_RINGPRED=1, g0 =
# GATHER=0, onelds = ONE_LDS=1); k_tb2 (fp64 increment form's kernel, tb2r2w4) under max-ilp
mkdir -p gpurun_out
tools/r4_ab_multi.sh 2 main:tb4:0 pred:tb4:0 g0:tb4:0 onelds:tb4:0 || exit 1
EXTRA="--math exact" tools/r4_ab_multi.sh 1 main:tb4:0 pred:tb4:0 g0:tb4:0 onelds:tb4:0 || exit 1
EXTRA="--math exact --scheme delta" tools/r4_ab_multi.sh 2 main:auto:0 tbilp:auto:0 tbilpns:auto:0 || exit 1
tools/r4_ab_multi.sh 1 main:tb2:0 tbilp:tb2:0 tbilpns:tb2:0 || exit 1
