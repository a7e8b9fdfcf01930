#!/bin/bash
# One rocprofv3 run per counter pass (the pool's rule: never several passes in one run, each
# under its own hard time limit), CSV output in gpurun_out/<tag>/pmc_<n>/, then the per-kernel
# summary of tools/pmc_summary.py.
#   tools/pmc_passes.sh <tag> <counter-file> <kernel-name-substring> -- <program args...>
# The program must be a binary or python3 directly (no env/bash hops under rocprofv3).
set -u
cd "$(dirname "$0")/.."
tag=$1; file=$2; match=$3; shift 3
[ "$1" = "--" ] && shift
out=$PWD/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
n=0
while read -r line; do
    case "$line" in pmc:*) ;; *) continue ;; esac
    n=$((n + 1))
    ctrs=${line#pmc:}
    echo "pass $n:$ctrs"
    timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv \
        -d "$out/pmc_$n" -o run -- "$@" > "$out/pass_$n.log" 2>&1
    st=$?
    if [ $st -ne 0 ]; then echo "pass $n failed with $st (see $out/pass_$n.log)"; exit $st; fi
done < "$file"
# rocprofv3 nests the CSVs under a host/pid directory: flatten to pmc_<n>/run_*.csv
for d in "$out"/pmc_*; do
    for f in $(find "$d" -name "run_*.csv"); do
        [ "$(dirname "$f")" = "$d" ] || mv "$f" "$d/"
    done
done
python3 tools/pmc_summary.py "$out" "$match" | tee "$out/summary.txt"
