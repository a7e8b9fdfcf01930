#!/bin/bash
# round 4: math / dtype A/B of tb3 vs tb4, then the full GPU suite, then the modelled-link overlap
mkdir -p gpurun_out
W=3d-wave-equation-mpi-cuda_amd/build/wave3d
for rep in 1 2; do
  for cfg in "tb3 exact fp64" "tb4 exact fp64" "tb3 fma fp32" "tb4 fma fp32"; do
    set -- $cfg
    echo -n "round=$rep $1 $2 $3 "
    timeout -k 10 120 $W 512 1 pi pi pi 1 100 --math $2 --dtype $3 --scheme leapfrog --kernel $1 --repeat 5 --warmup 1 \
        --json --quiet --format none \
      | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'])" || exit 1
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gputest_r4b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 tools/r4_overlap_model.sh 1 > gpurun_out/overlap_model.log 2>&1; echo "overlap rc=$?"; cat gpurun_out/overlap_model.log
