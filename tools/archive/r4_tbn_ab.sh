#!/bin/bash
# A/B of the deep-sweep load pipelines (WAVE3D_TBN_DEEP: bit 0 = A three planes ahead with A(i-1)
# from LDS, bit 1 = B two planes ahead) against k_tb3: N=512 fp64 K=100 --math fma, best of 5
# solves, alternating rounds. tools/archive/r4_tbn_ab.sh ROUNDS "kernel:deep ..."
cd "$(dirname "$0")/.."
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
rounds=$1; shift
for rep in $(seq "$rounds"); do
  for v in $*; do
    k=${v%%:*}; d=${v##*:}
    echo -n "round=$rep $k deep=$d "
    WAVE3D_TBN_DEEP=$d timeout -k 10 120 $W ${N:-512} 1 pi pi pi 1 ${K:-100} --math fma --kernel $k --repeat 5 --warmup 1 \
        --json --quiet --format none ${EXTRA:-} \
      | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'])" || exit 1
  done
done
