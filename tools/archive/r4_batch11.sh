#!/bin/bash
# round 4: GPU suite with the gather default and k_tb3's per-tile LDS objects; tb3 A/B (one LDS
# array vs per-tile objects) on config 5's kernel and fp64; bench.py
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4e.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gputest_r4e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r4e.json 2> gpurun_out/bench_r4e.err || exit 1
cat gpurun_out/bench_r4e.json
EXTRA="--math exact --dtype fp32 --scheme delta" tools/r4_ab_multi.sh 2 main:tb3:0 tb3one:tb3:0 || exit 1
N=2048 K=200 REP=2 TMO=240 EXTRA="--math exact --dtype fp32 --scheme delta" tools/r4_ab_multi.sh 1 main:tb3:0 tb3one:tb3:0 || exit 1
tools/r4_ab_multi.sh 2 main:tb3:0 tb3one:tb3:0 main:tb4:0 || exit 1
# tb4 memory ablations (wrong values, timing only): loads / stores / both pinned to one plane
tools/r4_ab_multi.sh 1 main:tb4:0 abl1:tb4:0 abl2:tb4:0 abl3:tb4:0 || true
