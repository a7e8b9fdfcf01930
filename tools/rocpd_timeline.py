#!/usr/bin/env python3
"""Stream timeline of a rocprofv3 --kernel-trace database: per HIP stream (queue) the busy time,
and how much of it ran while another stream was busy (concurrency), over the last solve.

    python tools/rocpd_timeline.py gpurun_out/trace_ov/ov_results.db
"""
import collections
import sqlite3
import subprocess
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main(path):
    c = sqlite3.connect(path)
    names = {k: n for k, n in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    rows = list(c.execute("select kernel_id, queue_id, stream_id, start, end, grid_size_x from rocpd_kernel_dispatch "
                          "order by start"))
    # the last solve: from the last k_init (the IC) to the end
    init_ids = {k for k, n in names.items() if "k_init" in n and "k_init_err" not in n}
    t0 = max(r[3] for r in rows if r[0] in init_ids)
    rows = [r for r in rows if r[3] >= t0]
    t1 = max(r[4] for r in rows)
    by = collections.defaultdict(list)
    kinds = collections.defaultdict(lambda: collections.Counter())
    for k, q, st, s, e, gx in rows:
        key = (q, st)
        by[key].append((s, e))
        nm = subprocess.run(["c++filt"], input=names[k], capture_output=True, text=True).stdout.strip()
        nm = nm.replace("wave3d::(anonymous namespace)::", "").split("(")[0]
        kinds[key][nm] += e - s
    span = t1 - t0
    keys = sorted(by)
    U = {k: union(v) for k, v in by.items()}
    print(f"last solve: {span / 1e6:.2f} ms, {len(rows)} dispatches")
    for k in keys:
        busy = sum(e - s for s, e in U[k])
        other = union([iv for kk in keys if kk != k for iv in U[kk]])
        conc = overlap(U[k], other)
        top = ", ".join(f"{n} {t / 1e6:.1f}" for n, t in kinds[k].most_common(4))
        print(f"queue {k[0]} stream {k[1]}: busy {busy / 1e6:.2f} ms ({100 * busy / span:.0f} %), "
              f"concurrent with the others {conc / 1e6:.2f} ms | {top}")
    allu = union([iv for v in U.values() for iv in v])
    print(f"GPU busy (any stream) {sum(e - s for s, e in allu) / 1e6:.2f} ms of {span / 1e6:.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
