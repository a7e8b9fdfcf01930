#!/bin/bash
# round 4: loopback halo copies of simulated ranks on the DMA engines (WAVE3D_LOOP_COPY=sdma,
# hipMemcpyDeviceToDeviceNoCU) vs HIP's copy kernels (blit), overlap off / on, zero-cost and
# modelled 50 GB/s links (tools/r4_overlap_model.sh), tb4 N=1024 K=100 fma
mkdir -p gpurun_out
for mode in blit sdma; do
  echo "== WAVE3D_LOOP_COPY=$mode"
  WAVE3D_LOOP_COPY=$mode P=2 DIMS=2,1,1 KER=tb4 tools/r4_overlap_model.sh 1 || exit 1
  WAVE3D_LOOP_COPY=$mode P=8 DIMS=2,2,2 KER=tb4 tools/r4_overlap_model.sh 1 || exit 1
done
for mode in blit sdma; do
  echo "== WAVE3D_LOOP_COPY=$mode (round 2)"
  WAVE3D_LOOP_COPY=$mode P=2 DIMS=2,1,1 KER=tb4 tools/r4_overlap_model.sh 1 || exit 1
  WAVE3D_LOOP_COPY=$mode P=8 DIMS=2,2,2 KER=tb4 tools/r4_overlap_model.sh 1 || exit 1
done
