#!/bin/bash
# RCCL CTA budget vs interior/shell overlap, one rank on one GPU with the periodic x wrap sent
# to itself through RCCL (--x-self-transport), N=512 fp64 K=100, tb2. WAVE3D_RCCL_MAX_CTAS=0
# is RCCL's default channel/CTA count. Prints one RESULT line per arm (mpts_per_s_best).
cd "$(dirname "$0")/.."
N=${N:-512}
K=${K:-tb2}
for ctas in ${CTAS:-0 1 2 4 8}; do
  for ov in "" "--no-overlap"; do
    echo -n "ctas=$ctas kernel=$K ov=${ov:-on} "
    WAVE3D_RCCL_MAX_CTAS=$ctas timeout -k 10 120 python3 tools/dist_solve.py --backend hip --transport rccl -- \
        $N 1 pi pi pi 1 100 --kernel $K --x-self-transport $ov --repeat 4 --warmup 1 | grep RESULT \
        | python3 -c "import sys,json; r=json.loads(sys.stdin.read()[7:]); print(round(r['mpts_per_s_best']), r['overlap'], r['comm_size'])" || exit 1
  done
done
echo -n "fused wrap (no transport): "
timeout -k 10 120 python3 bench.py --steps 4 --warmup 1 | python3 -c "import sys,json; print(round(json.loads(sys.stdin.read())['value']))"
