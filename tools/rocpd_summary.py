#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 (ROCm 7) ``*_results.db`` (rocpd SQLite output of
``--kernel-trace``): calls, total / mean duration, share, LDS, scratch (VGPRs: `make resources`).

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db [--width 90]
"""
import argparse
import sqlite3


def summarise(path, width=90):
    c = sqlite3.connect(path)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), max(lds_size),"
        " max(scratch_size) from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = ["kernel | calls | total_us | avg_us | pct | lds_B | scratch_B"]
    for name, n, tot, avg, lds, scr in rows:
        out.append(f"{name[:width]} | {n} | {tot / 1e3:.1f} | {avg / 1e3:.1f} | "
                   f"{100.0 * tot / total:.2f} | {lds} | {scr}")
    return "\n".join(out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--width", type=int, default=90)
    a = ap.parse_args()
    print(summarise(a.db, a.width))
