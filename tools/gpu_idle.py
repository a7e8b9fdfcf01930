#!/usr/bin/env python3
"""GPU busy/idle split of a rocprofv3 trace (rocpd SQLite `*_results.db`): the union of all
kernel (and memory-copy, when traced) intervals over all streams against the wall time from
the first to the last activity, plus the largest idle gaps. Separates "the overlap split costs
extra work" (busy time grows) from "dependencies leave the GPU idle" (gaps grow).

    python tools/gpu_idle.py gpurun_out/ovl_on/run_results.db [--top 5]
"""
import argparse
import sqlite3


def activity(db):
    c = sqlite3.connect(db)
    iv = [(s, e, n) for s, e, n in c.execute("select start, end, name from kernels")]
    try:
        iv += [(s, e, "copy") for s, e in c.execute("select start, end from memory_copies")]
    except sqlite3.Error:
        pass
    return sorted(iv)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=5)
    a = ap.parse_args()
    iv = activity(a.db)
    busy, gaps = 0, []
    cs, ce, prev_name = iv[0][0], iv[0][1], iv[0][2]
    for s, e, n in iv[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append((s - ce, prev_name, n))
            cs, ce = s, e
        elif e > ce:
            ce = e
        if e >= ce:
            prev_name = n
    busy += ce - cs
    wall = max(e for _, e, _ in iv) - iv[0][0]
    idle = sum(g for g, _, _ in gaps)
    print(f"activities {len(iv)}  wall {wall / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  "
          f"idle {idle / 1e6:.3f} ms ({100.0 * idle / wall:.1f} %) in {len(gaps)} gaps")
    short = lambda n: n.replace("(anonymous namespace)::", "").split("(")[0][-40:]
    for g, p, n in sorted(gaps, reverse=True)[: a.top]:
        print(f"  gap {g / 1e3:8.1f} us  after {short(p)}  before {short(n)}")


if __name__ == "__main__":
    main()
