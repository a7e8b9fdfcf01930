#!/bin/bash
# round 4: XCD block tile order vs bands for tb4; kernel-trace stats of bench.py; --fill-hbm 0.9 run
mkdir -p gpurun_out
tools/ab_env.sh WAVE3D_TILE_ORDER "band b" 3 -- 512 1 pi pi pi 1 100 --math fma --repeat 5 --warmup 1 \
  | python3 -c "
import sys, json
for l in sys.stdin:
    v, j = l.split(' ', 1); r = json.loads(j); print(v, round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'])" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4 -o bench -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_r4_bench.log 2>&1 || exit 1
tail -1 gpurun_out/prof_r4_bench.log
find gpurun_out/prof_r4 -name "*kernel_stats.csv" | head -1 | xargs head -8
timeout -k 10 400 python bench.py --fill-hbm 0.9 --timesteps 0 --steps 2 --warmup 1 > gpurun_out/bench_fill.json 2> gpurun_out/bench_fill.err || exit 1
cat gpurun_out/bench_fill.json
