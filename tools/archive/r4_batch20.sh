#!/bin/bash
# round 4: the max-ilp / max-memory-clause machine schedulers on k_tbn (fp64 and fp32 leapfrog),
# k_tb3 (config 5's fp32 increment form, fp64 fma), and max-ilp with deeper register prefetch
mkdir -p gpurun_out
tools/r4_ab_multi.sh 2 main:tb4:0 ilp:tb4:0 memc:tb4:0 ilpdeep:tb4:1 ilpdeep:tb4:2 || exit 1
EXTRA="--dtype fp32" tools/r4_ab_multi.sh 2 main:tb4:0 ilp:tb4:0 memc:tb4:0 || exit 1
EXTRA="--math exact --dtype fp32 --scheme delta" tools/r4_ab_multi.sh 2 main:tb3:0 tb3ilp:tb3:0 tb3memc:tb3:0 || exit 1
N=2048 K=200 REP=2 TMO=240 EXTRA="--math exact --dtype fp32 --scheme delta" tools/r4_ab_multi.sh 1 main:tb3:0 tb3ilp:tb3:0 tb3memc:tb3:0 || exit 1
tools/r4_ab_multi.sh 1 main:tb3:0 tb3ilp:tb3:0 tb3memc:tb3:0 || exit 1
