#!/bin/bash
# round 4: the fp32 increment form on four-layer sweeps (k_tbn DELTA): parity tests, then tb3 vs
# tb4 on config 5's scheme
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py -m gpu -x -q -k "delta" --timeout 300 --timeout-method thread > gpurun_out/gputest_delta.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gputest_delta.log; [ $rc -eq 0 ] || exit $rc
EXTRA="--math exact --dtype fp32 --scheme delta" tools/r4_ab_multi.sh 2 main:tb3:0 main:tb4:0 || exit 1
EXTRA="--dtype fp32 --scheme delta" tools/r4_ab_multi.sh 2 main:tb3:0 main:tb4:0 || exit 1
N=2048 K=200 REP=2 TMO=240 EXTRA="--math exact --dtype fp32 --scheme delta" tools/r4_ab_multi.sh 1 main:tb3:0 main:tb4:0 || exit 1
