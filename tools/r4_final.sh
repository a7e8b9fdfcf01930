#!/bin/bash
# round 4 final check: the GPU suite, smoke(), bench.py (fma, exact) on the committed tree
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gputest_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit 1
cat gpurun_out/bench_final.json
