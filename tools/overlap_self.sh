#!/bin/bash
# One rank, one GPU, RCCL transport with the periodic x wrap sent to itself (--x-self-transport):
# the real-launch cost of the interior/shell split + RCCL halo vs the same run without overlap
# and vs the fused local wrap. Prints one JSON line per configuration.
cd "$(dirname "$0")/.."
N=${N:-512}
for extra in "" "--no-overlap"; do
  for k in tb2 march2; do
    echo -n "selfsend kernel=$k ov=${extra:-on} "
    timeout -k 10 120 python3 tools/dist_solve.py --backend hip --transport rccl -- $N 1 pi pi pi 1 100 \
        --kernel $k --x-self-transport $extra --repeat 3 --warmup 1 | grep RESULT || exit 1
  done
done
