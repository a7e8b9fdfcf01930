#!/bin/bash
# round 4: every BASELINE config on one MI355X (multi-GPU configs as simulated ranks), exact and fma
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/run_baseline_configs.py --simulate --repeat 2 --math exact > gpurun_out/configs_exact.txt 2>&1 || exit 1
cat gpurun_out/configs_exact.txt
timeout -k 10 500 python -u tools/run_baseline_configs.py --simulate --repeat 2 --math fma --only gpu512 gpu512x2 gpu1024x4 gpu1024x8 gpu2048x8_fp32 > gpurun_out/configs_fma.txt 2>&1 || exit 1
cat gpurun_out/configs_fma.txt
