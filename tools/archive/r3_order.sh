#!/bin/bash
# Tile order (WAVE3D_TILE_ORDER 0 k-fastest, 1 j-fastest, 2 XCD bands) and non-temporal load
# ablations of the default fp64 fma tb3 sweep, N=512 K=100, best of 5 solves, 2 rounds.
cd "$(dirname "$0")/.."
for rep in 1 2; do
  for v in "cur:2" "cur:1" "cur:0" "abl5:2" "abl6:2"; do
    b=${v%%:*}; o=${v##*:}
    B=3d-wave-equation-mpi-cuda_amd/build/wave3d; [ $b != cur ] && B=gpurun_ab/$b/wave3d
    echo -n "rep=$rep build=$b order=$o: "
    WAVE3D_TILE_ORDER=$o timeout -k 10 120 $B 512 1 pi pi pi 1 100 --math fma --repeat 5 --warmup 1 --json --quiet --format none \
      | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'])" || exit 1
  done
done
