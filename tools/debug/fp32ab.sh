#!/bin/bash
# fp32 A/B of the tb4 sweep: leapfrog and increment form, fma and exact (ARMS = builds)
cd "$(dirname "$0")/../.."
A=${ARMS:-main old}
arms() { for b in $A; do echo -n "$b:$1:0 "; done; }
EXTRA="--dtype fp32" tools/r4_ab_multi.sh 2 $(arms tb4) > gpurun_out/ab_fp32_leap.txt 2>&1 || exit 1
EXTRA="--dtype fp32 --scheme delta" tools/r4_ab_multi.sh 2 $(arms tb4) main:tb3:0 > gpurun_out/ab_fp32_delta.txt 2>&1 || exit 1
EXTRA="--dtype fp32 --scheme delta --math exact" tools/r4_ab_multi.sh 2 $(arms tb4) main:tb3:0 > gpurun_out/ab_fp32_delta_exact.txt 2>&1
