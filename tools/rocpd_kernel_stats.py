#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 --kernel-trace database (the rocpd SQLite output that
rocprofv3 writes when no --output-format is given): calls, total / mean / share of GPU time,
registers and LDS per kernel symbol.

    python tools/rocpd_kernel_stats.py gpurun_out/prof_r4/bench_results.db [top]
"""
import collections
import sqlite3
import subprocess
import sys


def main(path, top=15):
    c = sqlite3.connect(path)
    sym = {}
    for kid, name, vg, ag, sg, lds in c.execute(
            "select id, kernel_name, arch_vgpr_count, accum_vgpr_count, sgpr_count, group_segment_size "
            "from rocpd_info_kernel_symbol"):
        sym[kid] = (name, vg, ag, sg, lds)
    t = collections.defaultdict(list)
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        t[kid].append(e - s)
    total = sum(sum(v) for v in t.values())
    names = [sym[k][0] for k in t]
    try:
        dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    except OSError:
        dem = names
    rows = sorted(((sum(v), len(v), k) for k, v in t.items()), reverse=True)
    print(f"{'share':>6} {'total ms':>10} {'calls':>6} {'mean us':>9} {'vgpr':>5} {'sgpr':>5} {'lds B':>7}  kernel")
    for tot, n, k in rows[:top]:
        name = dem[list(t).index(k)].replace("wave3d::(anonymous namespace)::", "")
        name = name.split("(")[0] if "(" in name else name
        _, vg, ag, sg, lds = sym[k]
        print(f"{100 * tot / total:5.1f}% {tot / 1e6:10.3f} {n:6d} {tot / n / 1e3:9.1f} {vg:5d} {sg:5d} {lds:7d}  {name}")
    print(f"total GPU kernel time {total / 1e6:.3f} ms over {sum(len(v) for v in t.values())} dispatches")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 15)
