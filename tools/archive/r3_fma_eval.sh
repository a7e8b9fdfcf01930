#!/bin/bash
# Round-3 evaluation of --math fma: chunk length of the fp64 default (tb3r1w8), fp32 accuracy /
# speed at N=512 and N=2048, the headline bench, then PMC passes of the fp64 sweep.
set -u
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
run() {  # N K dtype scheme kernel math chunk
  timeout -k 10 150 $B $1 1 pi pi pi 1 $2 --dtype $3 --scheme $4 --kernel $5 --math $6 ${7:+--chunk $7} \
      --repeat 5 --warmup 1 --json --quiet --format none \
    | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'], r['math'])"
}
for rep in 1 2; do
  for c in 64 96 128 171; do echo -n "fp64 N=512 tb3r1w8 fma chunk=$c: "; run 512 100 fp64 leapfrog tb3r1w8 fma $c || exit 1; done
done
for m in exact fma; do
  echo -n "fp32 N=512 leapfrog tb3 $m: "; run 512 100 fp32 leapfrog tb3 $m || exit 1
  echo -n "fp32 N=512 delta tb3 $m: "; run 512 100 fp32 delta tb3 $m || exit 1
  echo -n "fp32 N=2048 delta tb3 $m: "; run 2048 200 fp32 delta tb3 $m || exit 1
  echo -n "fp32 N=2048 leapfrog tb3 $m: "; run 2048 200 fp32 leapfrog tb3 $m || exit 1
done
echo "bench:"
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 || exit 1
