#!/bin/bash
# round 4: tb4 load-pipeline depth (WAVE3D_TBN_DEEP: bit 0 A three planes ahead, bit 1 B two ahead)
# on the current k_tbn, after the memory ablation showed the reads are what it waits for
mkdir -p gpurun_out
tools/r4_ab_multi.sh 3 main:tb4:0 deepv:tb4:1 deepv:tb4:2 deepv:tb4:3 || exit 1
