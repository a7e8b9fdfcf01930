#!/bin/bash
# round 4: k_tb3 (config 5's fp32 increment form) with raised wave priority during the prefetch
# (tb3p1), one LDS array per tile pair (tb3one), both; main = the tree
mkdir -p gpurun_out
EXTRA="--dtype fp32 --scheme delta --math exact" tools/r4_ab_multi.sh 2 main:tb3:0 tb3p1:tb3:0 tb3one:tb3:0 tb3both:tb3:0 || exit 1
EXTRA="--dtype fp32 --scheme delta" tools/r4_ab_multi.sh 1 main:tb3:0 tb3p1:tb3:0 tb3one:tb3:0 tb3both:tb3:0 || exit 1
N=2048 K=200 REP=2 TMO=240 EXTRA="--dtype fp32 --scheme delta --math exact" tools/r4_ab_multi.sh 1 main:tb3:0 tb3p1:tb3:0 tb3one:tb3:0 tb3both:tb3:0 || exit 1
