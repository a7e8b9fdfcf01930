#!/bin/bash
# Alternating A/B of gpurun_ab/<variant> builds over kernel/dtype/scheme/math arms:
#   ARMS="tb3:fp64:leapfrog:fma ..." tools/ab_r3_tiles.sh variant...
cd "$(dirname "$0")/.."
for arm in ${ARMS:-tb3:fp64:leapfrog:fma tb3r1w8:fp64:leapfrog:fma tb3:fp32:delta:fma tb3:fp32:delta:exact}; do
  IFS=: read k dt sc m <<< "$arm"
  for rep in 1 2; do
    for v in "$@"; do
      echo -n "$k $dt $sc $m $v: "
      timeout -k 10 120 gpurun_ab/$v/wave3d ${N:-512} 1 pi pi pi 1 ${K:-100} --kernel $k --dtype $dt --scheme $sc \
          --math $m --repeat 5 --warmup 1 --json --quiet --format none \
        | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'])" || exit 1
    done
  done
done
