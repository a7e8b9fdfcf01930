#!/bin/bash
# round 4: k_tbn kernel tests, tb4 solver tests, tb3 vs tb4 timing (N=512 fp64 fma K=100)
mkdir -p gpurun_out
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
timeout -k 10 300 python -u -m pytest tests/test_gpu_tb_kernels.py -x -q -k "tbn or fma" --timeout 120 --timeout-method thread > gpurun_out/tbn_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -3 gpurun_out/tbn_kernels.log; [ $rc -eq 0 ] || exit $rc
for k in tb3 tb4 tb3 tb4; do
  echo -n "$k fma "; timeout -k 10 120 $W 512 1 pi pi pi 1 100 --math fma --kernel $k --repeat 5 --warmup 1 --json --quiet --format none \
    | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'])" || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py -x -q -k "tb4" --timeout 300 --timeout-method thread > gpurun_out/tb4_solver.log 2>&1
rc=$?; echo "solver tests rc=$rc"; tail -15 gpurun_out/tb4_solver.log
