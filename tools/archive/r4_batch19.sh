#!/bin/bash
# round 4: k_tbn under the compiler's alternative machine schedulers (tools/ab_build.sh hip_tbn
# variants: ilp = max-ilp, memc = max-memory-clause, bias0 = schedule-metric-bias 0 (latency over
# occupancy), trk = AMDGPU register-pressure trackers); fp64 N=512 K=100
mkdir -p gpurun_out
tools/r4_ab_multi.sh 2 main:tb4:0 ilp:tb4:0 memc:tb4:0 bias0:tb4:0 trk:tb4:0 || exit 1
EXTRA="--math exact" tools/r4_ab_multi.sh 1 main:tb4:0 ilp:tb4:0 memc:tb4:0 bias0:tb4:0 trk:tb4:0 || exit 1
