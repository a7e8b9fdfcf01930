#!/bin/bash
# k_init variants: kernel time of layer 0 (rocprofv3 kernel stats), N=512 K=4, per build
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
for b in ${BUILDS:-main}; do
  W=gpurun_ab/$b/wave3d; [ "$b" = main ] && W=3d-wave-equation-mpi-cuda_amd/build/wave3d
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/init_$b -o run -- $W 512 1 pi pi pi 0.04 4 --math fma --repeat 5 --quiet --format none > /dev/null 2>&1 || exit 1
  echo "== $b"; python3 tools/rocpd_kernel_stats.py gpurun_out/init_$b/run_results.db | grep -E "k_init<"
done
