#!/usr/bin/env python3
"""Concurrency of kernels on different HIP streams in a rocprofv3 kernel trace (rocpd SQLite
`*_results.db`): for every pair of streams, the wall time during which kernels of both run,
against each stream's busy time. Shows that the interior sweep (compute stream) overlaps the
shells / halo kernels (comm stream).

    python tools/stream_overlap.py gpurun_out/prof/run_results.db
"""
import argparse
import collections
import sqlite3


def intervals(db):
    c = sqlite3.connect(db)
    rows = c.execute("select stream_id, start, end, name from kernels order by start").fetchall()
    per = collections.defaultdict(list)
    names = collections.defaultdict(collections.Counter)
    for sid, s, e, n in rows:
        per[sid].append((s, e))
        short = n.replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
        names[sid][short.split("::")[-1].replace("void ", "")[:24]] += 1
    return per, names


def union(iv):
    out = []
    for s, e in sorted(iv):
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
        if s < e:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    a = ap.parse_args()
    per, names = intervals(a.db)
    u = {k: union(v) for k, v in per.items()}
    busy = {k: sum(e - s for s, e in v) for k, v in u.items()}
    for k in sorted(u):
        top = ", ".join(f"{n} x{c}" for n, c in names[k].most_common(4))
        print(f"stream {k}: busy {busy[k] / 1e6:.2f} ms, kernels: {top}")
    ks = sorted(u)
    for x in range(len(ks)):
        for y in range(x + 1, len(ks)):
            ov = overlap(u[ks[x]], u[ks[y]])
            if ov:
                print(f"streams {ks[x]} & {ks[y]}: both running {ov / 1e6:.2f} ms "
                      f"({100 * ov / busy[ks[y]]:.0f} % of stream {ks[y]}'s busy time)")
