#!/bin/bash
# PMC passes of the tb3 tiles (fp64 N=512 K=40), one rocprofv3 run per pass.
#   tools/pmc_tb3.sh [kernels...]   (default: tb3r1w8 tb3)
set -e
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
ks=${*:-tb3r1w8 tb3}
for k in $ks; do
    tools/pmc_passes.sh pmc_$k tools/pmc_tb.txt k_tb3 -- $B 512 1 pi pi pi 1 40 --kernel $k --quiet --format none
done
