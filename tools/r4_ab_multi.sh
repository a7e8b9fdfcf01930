#!/bin/bash
# Alternating A/B over builds and kernels: entries "build:kernel:deep", build = main (the tree's
# build/) or a gpurun_ab/<name> variant; N=512 fp64 K=100 --math fma, best of 5 solves.
#   tools/r4_ab_multi.sh ROUNDS main:tb3:0 split:tb4:0 ...
cd "$(dirname "$0")/.."
rounds=$1; shift
for rep in $(seq "$rounds"); do
  for v in "$@"; do
    IFS=: read -r b k d <<< "$v"
    W=gpurun_ab/$b/wave3d; [ "$b" = main ] && W=3d-wave-equation-mpi-cuda_amd/build/wave3d
    echo -n "round=$rep $b $k deep=$d "
    WAVE3D_TBN_DEEP=$d timeout -k 10 ${TMO:-120} $W ${N:-512} 1 pi pi pi 1 ${K:-100} --math fma --kernel $k --repeat ${REP:-5} --warmup 1 \
        --json --quiet --format none ${EXTRA:-} \
      | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.17g' % r['linf_abs'], '%.17g' % r['max_rel_final'], r['kernel'])" || exit 1
  done
done
