#!/bin/bash
# round 4: fp64 increment form (auto = tb2r2w4) vs tb3 / tb2r2w8 after this round's tb3 changes
mkdir -p gpurun_out
EXTRA="--scheme delta --math exact" tools/r4_ab_multi.sh 2 main:auto:0 main:tb3:0 main:tb2r2w8:0 || exit 1
EXTRA="--scheme delta" tools/r4_ab_multi.sh 2 main:auto:0 main:tb3:0 main:tb2r2w8:0 || exit 1
