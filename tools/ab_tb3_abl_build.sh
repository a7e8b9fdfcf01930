#!/bin/bash
# Builds timing-ablation variants of hip_tb3.hip (W3D_TB3_ABL=n, see the top of the file) into
# gpurun_ab/abl<n>/{libwave3d.so,wave3d}, linked against the tree's other objects (make first).
#   tools/ab_tb3_abl_build.sh 0 1 2 3
set -e
cd "$(dirname "$0")/../3d-wave-equation-mpi-cuda_amd"
ROCM=/opt/rocm
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unknown-pragmas --offload-arch=gfx950 -fopenmp -munsafe-fp-atomics -I$ROCM/include -Wno-pass-failed"
objs=$(ls build/hip/*.o | grep -v '/hip_tb3.o$')
for n in "$@"; do
  (
    out=../gpurun_ab/abl$n; mkdir -p $out
    $ROCM/bin/hipcc $FLAGS -DW3D_TB3_ABL=$n -c csrc/hip_tb3.hip -o $out/hip_tb3.o
    $ROCM/bin/hipcc -shared --offload-arch=gfx950 $objs $out/hip_tb3.o -L$ROCM/lib -lamdhip64 -lrccl \
        -lrocprofiler-sdk-roctx -fopenmp -Wl,-rpath,$ROCM/lib -o $out/libwave3d.so
    rm $out/hip_tb3.o
    cp build/wave3d $out/
    echo "built $out"
  ) &
done
wait
