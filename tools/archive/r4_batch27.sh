#!/bin/bash
# round 4: wave priority raised while a tb4 plane's prefetch loads issue (W3D_TBN_PRIO 1 / 3) vs the
# same build without (same = tools/ab_build.sh control) and the tree (main); fp64 fma / exact, fp32
mkdir -p gpurun_out
tools/r4_ab_multi.sh 2 main:tb4:0 same:tb4:0 prio1:tb4:0 prio3:tb4:0 || exit 1
EXTRA="--math exact" tools/r4_ab_multi.sh 1 main:tb4:0 prio1:tb4:0 prio3:tb4:0 || exit 1
EXTRA="--dtype fp32" tools/r4_ab_multi.sh 1 main:tb4:0 prio1:tb4:0 prio3:tb4:0 || exit 1
