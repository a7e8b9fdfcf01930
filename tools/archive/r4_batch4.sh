#!/bin/bash
# round 4: k_tb3 loop split A/B (main = split, tb3old = one loop) and tb4, fp64 fma / exact and the
# fp32 increment form (config 5's kernel, scalar noslp build vs the SLP-packed main build); then
# the GPU suite and the modelled-link overlap study
mkdir -p gpurun_out
set -o pipefail
A=tools/r4_ab_multi.sh
$A 2 main:tb3:0 tb3old:tb3:0 main:tb4:0 tb3old:tb4:0 || exit 1
EXTRA="--math exact" $A 2 main:tb3:0 tb3old:tb3:0 main:tb4:0 || exit 1
EXTRA="--math exact --dtype fp32 --scheme delta" $A 2 main:auto:0 tb3old:auto:0 noslp:auto:0 || exit 1
N=2048 K=200 REP=2 TMO=240 EXTRA="--math exact --dtype fp32 --scheme delta" $A 1 main:auto:0 tb3old:auto:0 noslp:auto:0 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gputest_r4b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 tools/r4_overlap_model.sh 1 > gpurun_out/overlap_model.log 2>&1; echo "overlap rc=$?"; cat gpurun_out/overlap_model.log
