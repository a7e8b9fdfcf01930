#!/bin/bash
# Alternating timing runs of gpurun_ab/<variant>/wave3d builds at the headline config
# (N=512 fp64 K=100, default kernel): tools/ab_tb3_abl.sh ROUNDS variant...
cd "$(dirname "$0")/.."
rounds=$1; shift
for rep in $(seq "$rounds"); do
  for v in "$@"; do
    echo -n "round=$rep $v "
    timeout -k 10 120 gpurun_ab/$v/wave3d ${N:-512} 1 pi pi pi 1 ${K:-100} --math fma --repeat 5 --warmup 1 \
        --json --quiet --format none ${EXTRA:-} \
      | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'])" || exit 1
  done
done
