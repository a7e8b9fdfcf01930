#!/bin/bash
# Round 5: the driver's 1/2/4/8-GPU bench commands rehearsed on ONE MI355X (n processes sharing
# the GPU through the staged transport; RCCL refuses duplicate GPUs), each at its BASELINE config
# and golden, with zero-cost halos and with an xGMI-like link model (--model-link 50,5), so the
# --overlap auto arm kept under each is on record. Warm-up 7 = the six trial solves + 1.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/scale_rehearsal_r5.jsonl
: > $out
for n in 1 2 4 8; do
  for link in "" "50,5"; do
    [ $n = 1 ] && [ -n "$link" ] && continue
    extra=""; [ -n "$link" ] && extra="--model-link $link"
    echo "== n=$n link=${link:-none}"
    timeout -k 10 600 python bench.py --gpus $n --steps 2 --warmup 7 --transport staged --shared-device $extra \
        > gpurun_out/rehearse_${n}_${link:-0}.json 2> gpurun_out/rehearse_${n}_${link:-0}.err || exit $?
    tail -1 gpurun_out/rehearse_${n}_${link:-0}.json | tee -a $out
  done
done
