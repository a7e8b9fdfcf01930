#!/bin/bash
# round 4: overlap with a CU-masked compute stream (WAVE3D_COMM_CUS CUs left to the halo stream),
# modelled 50 GB/s links, direct launches (a replayed graph drops stream CU masks)
mkdir -p gpurun_out
for cus in 0 8 16; do
  WAVE3D_COMM_CUS=$cus P=2 DIMS=2,1,1 KER=tb4 XARGS="--graph off" timeout -k 10 400 tools/r4_overlap_model.sh 1 | sed "s/^/cus=$cus /" || exit 1
done
for cus in 0 8 16; do
  WAVE3D_COMM_CUS=$cus KER=tb4 XARGS="--graph off" timeout -k 10 400 tools/r4_overlap_model.sh 1 | sed "s/^/cus=$cus /" || exit 1
done
