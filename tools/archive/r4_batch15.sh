#!/bin/bash
# round 4: shells-first overlap order (WAVE3D_OVERLAP_SHELLS_FIRST=1): parity, then the modelled-link
# overlap study against the default order on the same box
mkdir -p gpurun_out
WAVE3D_OVERLAP_SHELLS_FIRST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py -m gpu -x -q -k "overlap or decomposition or delta_fp32_matches" --timeout 300 --timeout-method thread > gpurun_out/gputest_sf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gputest_sf.log; [ $rc -eq 0 ] || exit $rc
for sf in 0 1; do
  WAVE3D_OVERLAP_SHELLS_FIRST=$sf P=2 DIMS=2,1,1 KER=tb4 timeout -k 10 400 tools/r4_overlap_model.sh 1 | sed "s/^/sf=$sf /" || exit 1
  WAVE3D_OVERLAP_SHELLS_FIRST=$sf KER=tb4 timeout -k 10 400 tools/r4_overlap_model.sh 1 | sed "s/^/sf=$sf /" || exit 1
done
