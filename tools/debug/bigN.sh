#!/bin/bash
# single-rank solves at sizes where a tile column's x range splits into several work items
cd "$(dirname "$0")/../.."
for N in ${NS:-1024}; do
  for b in ${BUILDS:-main old}; do
    W=gpurun_ab/$b/wave3d; [ "$b" = main ] && W=3d-wave-equation-mpi-cuda_amd/build/wave3d
    for m in ${MATHS:-fma}; do
      echo -n "N=$N $b $m "
      timeout -k 10 300 $W $N 1 pi pi pi 1 ${K:-100} --math $m --kernel ${KER:-auto} --json --quiet --format none \
        | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'])" || exit 1
    done
  done
done
