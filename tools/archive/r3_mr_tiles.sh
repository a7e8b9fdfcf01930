#!/bin/bash
# Simulated multi-rank bench configs (one GPU, loopback halos) for a list of fp64 fma kernels,
# overlap off: tools/archive/r3_mr_tiles.sh tb3r1w8 tb3 ...
cd "$(dirname "$0")/.."
B=${BIN:-3d-wave-equation-mpi-cuda_amd/build/wave3d}
for k in "$@"; do
  for cfg in 512:2:2,1,1 1024:4:2,2,1 1024:8:2,2,2; do
    IFS=: read n r d <<< "$cfg"
    echo -n "N=$n ranks=$r dims=$d kernel=$k: "
    timeout -k 10 200 $B $n 1 pi pi pi 1 100 --ranks $r --dims $d --kernel $k --math fma --overlap ${OV:-off} \
        --repeat 3 --warmup 1 --json --quiet --format none \
      | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'], round(r['exchange_ms'],1))" || exit 1
  done
done
