#!/bin/bash
# Kernel traces of the simulated 2x2x2 N=1024 run (8 ranks on one GPU) with and without the
# interior/shell overlap, then busy/idle split (tools/gpu_idle.py) and per-kernel stats.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
B=3d-wave-equation-mpi-cuda_amd/build/wave3d
for o in on off; do
    extra=""; [ $o = off ] && extra="--no-overlap"
    timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/ovl_$o -o run -- \
        $B 1024 8 pi pi pi 1 20 --ranks 8 --dims 2,2,2 $extra --quiet --format none > gpurun_out/ovl_$o.log 2>&1
    db=$(find gpurun_out/ovl_$o -name "*_results.db" | head -1)
    echo "== overlap $o"; python3 tools/gpu_idle.py "$db" --top 8
    python3 tools/rocpd_summary.py "$db" | head -12
done
