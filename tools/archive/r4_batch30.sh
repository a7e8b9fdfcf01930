#!/bin/bash
# round 4: fp32 exact tb4 (645k now, 825k in batch 5): masks as products (mm0 = MASKMUL 0), one LDS
# array (onelds), predicated ring (pred1)
mkdir -p gpurun_out
EXTRA="--dtype fp32 --math exact" tools/r4_ab_multi.sh 2 main:tb4:0 mm0:tb4:0 onelds:tb4:0 pred1:tb4:0 || exit 1
EXTRA="--dtype fp32" tools/r4_ab_multi.sh 1 main:tb4:0 mm0:tb4:0 onelds:tb4:0 pred1:tb4:0 || exit 1
