#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 700 tools/archive/r4_batch7.sh > gpurun_out/overlap_cus.log 2>&1; rc=$?; cat gpurun_out/overlap_cus.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 480 tools/archive/r4_pmc2.sh > gpurun_out/pmc_r4b.log 2>&1; rc=$?; cat gpurun_out/pmc_r4b.log; exit $rc
