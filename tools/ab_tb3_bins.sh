#!/bin/bash
# Same-box A/B of the previous build (gpurun_ab/old) and the tree's build for the tb3 changes.
set -e
cd "$(dirname "$0")/.."
tools/ab_bins.sh 3 -- 512 1 pi pi pi 1 100 --dtype fp32 --warmup 1 --repeat 3 > gpurun_out/abbin_fp32_512.log
tools/ab_bins.sh 3 -- 512 1 pi pi pi 1 100 --kernel tb3r1w8 --warmup 1 --repeat 3 > gpurun_out/abbin_fp64_tb3r1w8.log
tools/ab_bins.sh 2 -- 2048 1 pi pi pi 1 200 --dtype fp32 --warmup 1 --repeat 2 > gpurun_out/abbin_fp32_2048.log
