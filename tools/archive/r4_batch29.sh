#!/bin/bash
# round 4: fp32 exact tb4 at 636k vs 825k in batch 5 -- which change: max-ilp (noilp), GATHER=1
# (noilpg0 / ilpg0)?
mkdir -p gpurun_out
EXTRA="--dtype fp32 --math exact" tools/r4_ab_multi.sh 2 main:tb4:0 noilp:tb4:0 noilpg0:tb4:0 ilpg0:tb4:0 prio1:tb4:0 || exit 1
EXTRA="--dtype fp32" tools/r4_ab_multi.sh 1 main:tb4:0 noilp:tb4:0 noilpg0:tb4:0 ilpg0:tb4:0 || exit 1
EXTRA="--math exact" tools/r4_ab_multi.sh 1 main:tb4:0 noilp:tb4:0 noilpg0:tb4:0 ilpg0:tb4:0 || exit 1
