#!/bin/bash
# Build A/B variants of HIP sources with extra compiler flags into gpurun_ab/<name>/
# {libwave3d.so, wave3d}, linked against the tree's other objects (make first):
#   tools/ab_build.sh hip_tb3 "nb2:-DW3D_TB3_NB=2" "nb4:-DW3D_TB3_NB=4"
#   tools/ab_build.sh hip_tb3,hip_tbn "noslp:-fno-slp-vectorize"
set -e
cd "$(dirname "$0")/../3d-wave-equation-mpi-cuda_amd"
ROCM=/opt/rocm
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unknown-pragmas --offload-arch=gfx950 -fopenmp -munsafe-fp-atomics -I$ROCM/include -Wno-pass-failed"
srcs=${1//,/ }; shift
# hip_tbn_exact.hip includes hip_tbn.hip (the --math exact kernels): a hip_tbn variant rebuilds both
case " $srcs " in *" hip_tbn "*) case " $srcs " in *" hip_tbn_exact "*) ;; *) srcs="$srcs hip_tbn_exact";; esac;; esac
objs=$(ls build/hip/*.o)
for src in $srcs; do objs=$(echo "$objs" | grep -v "/$src.o\$"); done
for v in "$@"; do
  (
    name=${v%%:*}; extra=${v#*:}
    out=../gpurun_ab/$name; mkdir -p $out
    vobjs=""
    for src in $srcs; do
      # the Makefile's per-object flags (NOSLP_OBJS), so a baseline arm builds the shipped code
      obj_flags=$(make -s -n build/hip/$src.o -W csrc/$src.hip 2>/dev/null | grep -o -- '-fno-slp-vectorize -mllvm -amdgpu-sched-strategy=[a-z-]*' | head -1)
      [ -n "${AB_NO_OBJ_FLAGS:-}" ] && obj_flags=""
      $ROCM/bin/hipcc $FLAGS $obj_flags $extra -c csrc/$src.hip -o $out/$src.o
      vobjs="$vobjs $out/$src.o"
    done
    $ROCM/bin/hipcc -shared --offload-arch=gfx950 $objs $vobjs -L$ROCM/lib -lamdhip64 -lrccl \
        -lrocprofiler-sdk-roctx -fopenmp -Wl,-rpath,$ROCM/lib -o $out/libwave3d.so
    rm $vobjs
    cp build/wave3d $out/
    echo "built $out"
  ) &
done
wait
