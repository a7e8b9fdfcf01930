#!/bin/bash
# round 4: GPU suite with tb4 as the leapfrog default, then the driver's bench (fma and exact)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gputest_r4c.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r4c.json 2> gpurun_out/bench_r4c.err || exit 1
cat gpurun_out/bench_r4c.json
timeout -k 10 300 python bench.py --math exact > gpurun_out/bench_r4c_exact.json 2> gpurun_out/bench_r4c_exact.err || exit 1
cat gpurun_out/bench_r4c_exact.json
