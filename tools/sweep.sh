#!/bin/bash
# Kernel-variant / chunk sweep of the single-GPU solve (N=512, K=100 unless overridden).
# Prints one JSON summary per configuration.  usage: tools/sweep.sh [N] [K] [dtype]
N=${1:-512}; K=${2:-100}; DT=${3:-fp64}
B="$(dirname "$0")/../3d-wave-equation-mpi-cuda_amd/build/wave3d"
for k in ${KERNELS:-march4 march2 march8 march4nt march2nt naive}; do
    for c in ${CHUNKS:-0 32 64 128 257}; do
        if [ "$k" = naive ] && [ "$c" != 0 ]; then continue; fi
        echo -n "$k chunk=$c "
        "$B" "$N" 1 pi pi pi 1 "$K" --dtype "$DT" --kernel "$k" --chunk "$c" --repeat 5 \
            --warmup 1 --json --format none --quiet || exit $?
    done
done
