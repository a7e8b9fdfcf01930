#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tb_kernels.py -m gpu -x -q -k "tbn" --timeout 300 --timeout-method thread > gpurun_out/gputest_tbnk.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/gputest_tbnk.log; exit $rc
