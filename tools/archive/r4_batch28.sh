#!/bin/bash
# round 4: confirm W3D_TBN_PRIO=1 on the fp32 tb4 sweep (batch 27: +2.5 % on one sample)
mkdir -p gpurun_out
EXTRA="--dtype fp32" tools/r4_ab_multi.sh 3 main:tb4:0 prio1:tb4:0 || exit 1
EXTRA="--dtype fp32 --math exact" tools/r4_ab_multi.sh 2 main:tb4:0 prio1:tb4:0 || exit 1
N=1024 K=100 REP=3 EXTRA="--dtype fp32" tools/r4_ab_multi.sh 1 main:tb4:0 prio1:tb4:0 || exit 1
