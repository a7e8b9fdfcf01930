#!/bin/bash
# round 4: face masks as products (mm) and SLP vectorisation off (noslp) over the deep sweeps
mkdir -p gpurun_out
A=tools/r4_ab_multi.sh
$A 2 main:tb4:0 mm:tb4:0 noslp:tb4:0 mmnoslp:tb4:0 main:tb3:0 mm:tb3:0 || exit 1
EXTRA="--math exact" $A 2 main:tb4:0 mm:tb4:0 mmnoslp:tb4:0 || exit 1
EXTRA="--dtype fp32 --scheme delta" $A 2 main:tb3:0 noslp:tb3:0 || exit 1
EXTRA="--dtype fp32 --scheme leapfrog" $A 2 main:tb3:0 noslp:tb3:0 main:tb4:0 noslp:tb4:0 mmnoslp:tb4:0 || exit 1
EXTRA="--math exact --dtype fp32 --scheme leapfrog" $A 1 main:tb3:0 noslp:tb3:0 noslp:tb4:0 || exit 1
P=2 DIMS=2,1,1 KER=tb4 timeout -k 10 500 tools/r4_overlap_model.sh 1 || exit 1
KER=tb4 timeout -k 10 500 tools/r4_overlap_model.sh 1 || exit 1
KER=tb4 XARGS="--chunk 128" timeout -k 10 500 tools/r4_overlap_model.sh 1 || exit 1
