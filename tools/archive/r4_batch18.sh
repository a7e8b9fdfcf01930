#!/bin/bash
# round 4: k_tb3 with the j neighbours of a wave's own rows from registers (W3D_TB3_JREG=1, the
# tree) vs LDS (nojreg): tb3 parity tests, then config 5's kernel (fp32 increment form) and fp64
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_tb_kernels.py -m gpu -x -q -k "tb3 or delta or fma" --timeout 300 --timeout-method thread > gpurun_out/gputest_jreg.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gputest_jreg.log; [ $rc -eq 0 ] || exit $rc
EXTRA="--math exact --dtype fp32 --scheme delta" tools/r4_ab_multi.sh 2 main:tb3:0 nojreg:tb3:0 || exit 1
EXTRA="--dtype fp32 --scheme delta" tools/r4_ab_multi.sh 2 main:tb3:0 nojreg:tb3:0 || exit 1
N=2048 K=200 REP=2 TMO=240 EXTRA="--math exact --dtype fp32 --scheme delta" tools/r4_ab_multi.sh 1 main:tb3:0 nojreg:tb3:0 || exit 1
tools/r4_ab_multi.sh 2 main:tb3:0 nojreg:tb3:0 || exit 1
EXTRA="--math exact" tools/r4_ab_multi.sh 1 main:tb3:0 nojreg:tb3:0 || exit 1
