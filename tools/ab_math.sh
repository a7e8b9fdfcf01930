#!/bin/bash
# fp64 kernel / stencil-arithmetic A/B at the headline config (N=512 K=100, one GPU): exact
# (reference operation order, bitwise) vs --math fma (coef/h^2 folded), tb2 vs tb3 tiles.
# Arms alternated over rounds; best of 5 solves per run; L-inf printed to check the golden.
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
N=${N:-512}
K=${K:-100}
DT=${DT:-fp64}
ARMS=${ARMS:-"tb2r2w8:exact tb2r2w8:fma tb3:exact tb3r1w8:exact tb3:fma tb3r1w8:fma tb3r1w16:fma"}
for rep in $(seq ${ROUNDS:-2}); do
  for arm in $ARMS; do
    k=${arm%%:*}; m=${arm##*:}
    echo -n "round=$rep kernel=$k math=$m "
    timeout -k 10 120 $B $N 1 pi pi pi 1 $K --dtype $DT --scheme ${SCHEME:-leapfrog} --kernel $k --math $m --repeat 5 --warmup 1 --json --quiet \
        --format none | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'], r['math'])" || exit 1
  done
done
