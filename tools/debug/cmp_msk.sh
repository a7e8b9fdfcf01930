#!/bin/bash
# first K (same dt as the N=512 K=100 golden run) at which two builds' exact errors part
cd "$(dirname "$0")/../.."
for K in ${KS:-4 8 12 16 24 32 48 64 100}; do
  T=$(python3 -c "print($K/100)")
  for b in ${BUILDS:-old msk}; do
    W=gpurun_ab/$b/wave3d
    echo -n "K=$K $b "
    timeout -k 10 60 $W 512 1 pi pi pi $T $K --math exact --kernel tb4 --json --quiet --format none | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print('%.17g %.17g' % (r['linf_abs'], r['max_rel_final']))" || exit 1
  done
done
