#!/bin/bash
# Simulated multi-rank runs on one GPU (loopback D2D halos, hipGraph): the bench's 2/4/8-rank
# configs with the fp64 kernels and both arithmetic forms, overlap on and off. Mpts/s best of 3.
cd "$(dirname "$0")/.."
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
run() {  # N ranks dims kernel math overlap
  timeout -k 10 200 $B $1 1 pi pi pi 1 100 --ranks $2 --dims $3 --kernel $4 --math $5 --overlap $6 \
      --repeat 3 --warmup 1 --json --quiet --format none \
    | python3 -c "import sys,json; r=json.loads(sys.stdin.read().splitlines()[-1]); print(round(r['mpts_per_s_best']), '%.9g' % r['linf_abs'], r['kernel'], r['math'], r['overlap'], round(r['exchange_ms'],1))"
}
for cfg in "512 2 2,1,1" "1024 4 2,2,1" "1024 8 2,2,2"; do
  set -- $cfg
  for km in ${KMS:-"auto fma" "tb2r2w8 fma" "tb2r2w8 exact"}; do
    for ov in on off; do
      echo -n "N=$1 ranks=$2 dims=$3 $km overlap=$ov: "
      run $1 $2 $3 $km $ov || exit 1
    done
  done
done
