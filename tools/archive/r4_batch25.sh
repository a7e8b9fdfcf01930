#!/bin/bash
# round 4: bench.py --math exact and --fill-hbm 0.9 on the max-ilp build; rocprofv3 kernel stats
# of bench.py (fma)
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --math exact > gpurun_out/bench_ilp_exact.json 2> gpurun_out/bench_ilp_exact.err || exit 1
cat gpurun_out/bench_ilp_exact.json
timeout -k 10 400 python bench.py --fill-hbm 0.9 --timesteps 0 --steps 2 --warmup 1 > gpurun_out/bench_ilp_fill.json 2> gpurun_out/bench_ilp_fill.err || exit 1
cat gpurun_out/bench_ilp_fill.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ilp -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_ilp.log 2>&1 || exit 1
tail -1 gpurun_out/prof_ilp.log
