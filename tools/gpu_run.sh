#!/bin/bash
# Sequential GPU steps for one gpurun call. Each step has its own time limit; the script
# stops at the first crash / abort / timeout (exit 124, 134, 137, 139) so nothing else
# touches a GPU that may be in a bad state. Ordinary test failures (exit 1) continue.
#   tools/gpu_run.sh "<name>:<seconds>:<command>" ...
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
    name="${spec%%:*}"; rest="${spec#*:}"
    secs="${rest%%:*}"; cmd="${rest#*:}"
    echo "=== [$name] (${secs}s) $cmd" | tee -a gpurun_out/steps.log
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    st=$?
    echo "=== [$name] exit=$st after $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
    tail -n 25 "gpurun_out/$name.log"
    case $st in
        124|134|137|139) echo "stopping: step $name ended with $st"; exit $st ;;
    esac
done
exit 0
