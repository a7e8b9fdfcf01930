#!/bin/bash
# round 4: XCD tile orders for tb4, measured properly (batch 13's "band b" arms both parsed as
# blocks): band (the default) vs blocks (4 x 2 XCD blocks) vs j; fp64 fma N=512 / N=1024, fp32
mkdir -p gpurun_out
summ() { python3 -c "
import sys, json
for l in sys.stdin:
    v, j = l.split(' ', 1); r = json.loads(j); print(v, round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'])"; }
tools/ab_env.sh WAVE3D_TILE_ORDER "band blocks j" 2 -- 512 1 pi pi pi 1 100 --math fma --repeat 5 --warmup 1 | summ || exit 1
tools/ab_env.sh WAVE3D_TILE_ORDER "band blocks" 1 -- 1024 1 pi pi pi 1 40 --math fma --repeat 3 --warmup 1 | summ || exit 1
tools/ab_env.sh WAVE3D_TILE_ORDER "band blocks" 2 -- 512 1 pi pi pi 1 100 --math fma --dtype fp32 --repeat 5 --warmup 1 | summ || exit 1
