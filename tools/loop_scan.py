#!/usr/bin/env python3
"""Loops of one kernel in a gfx950 device assembly file: for every backward branch, the
instruction mix of the region it closes (VALU, LDS, LDS-DMA pieces, SGPR-spill reloads,
scratch, s_waitcnt) — the steady plane loop of a sweep is the largest one.

    python tools/loop_scan.py /tmp/tbn.s 'k_tbnIdLi4ELb0ELi2ELi8ELb1ELb0E'
"""
import collections
import re
import sys


def main(path, filt):
    text = open(path).read()
    for m in re.finditer(r"\n(_Z[^\s:]*" + re.escape(filt) + r"[^\s:]*):", text):
        name = m.group(1)
        start = text.find("\n", m.end()) + 1
        end = text.find(".Lfunc_end", start)
        lines = [l.strip() for l in text[start:end].split("\n")]
        labels = {}
        for n, l in enumerate(lines):
            mm = re.match(r"^(\.LBB[^\s:]+):", l)
            if mm:
                labels[mm.group(1)] = n
        print(name)
        for n, l in enumerate(lines):
            mm = re.match(r"^s_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
            if not mm or mm.group(2) not in labels or labels[mm.group(2)] > n:
                continue
            body = lines[labels[mm.group(2)]:n + 1]
            c = collections.Counter()
            for t in body:
                if not t or t[0] in ";." or t.endswith(":"):
                    continue
                op = t.split()[0]
                c[op] += 1
                if op.startswith("buffer_load") and t.endswith(" lds"):
                    c["dma"] += 1
                if op == "s_waitcnt" and "vmcnt" in t:
                    c["vmwait"] += 1
            tot = sum(v for k, v in c.items() if k not in ("dma", "vmwait"))
            valu = sum(v for k, v in c.items() if k.startswith("v_"))
            lds = sum(v for k, v in c.items() if k.startswith("ds_"))
            scr = sum(v for k, v in c.items() if k.startswith("scratch_"))
            print("  loop %-14s lines %5d  insts %5d  valu %5d  lds %4d  dma %3d  readlane %4d  writelane %4d  "
                  "scratch %3d  vmcnt-waits %3d  barriers %3d" %
                  (mm.group(2), n - labels[mm.group(2)], tot, valu, lds, c["dma"], c["v_readlane_b32"],
                   c["v_writelane_b32"], scr, c["vmwait"], c["s_barrier"]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
