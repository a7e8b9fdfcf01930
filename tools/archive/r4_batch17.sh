#!/bin/bash
# round 4: three-arm --overlap auto (on beside / off / on shells first): the trial tests, the bench
# multi-process paths, the overlap parity tests
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_halo_selftest.py tests/test_bench.py tests/test_dist.py tests/test_gpu_solver.py -m gpu -x -q -k "overlap or bench or dist or rccl or multiprocess" --timeout 300 --timeout-method thread > gpurun_out/gputest_3arm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/gputest_3arm.log; exit $rc
