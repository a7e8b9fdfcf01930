#!/usr/bin/env python3
"""Per-kernel resource summary of a gfx950 device assembly file (hipcc --cuda-device-only -S).

For every kernel whose (mangled) name contains FILTER: VGPRs, AGPRs, SGPRs, spills, LDS,
scratch, and instruction counts that matter to the stencil sweeps (VALU, packed fp32 v_pk_*,
v_readlane/v_writelane = SGPR spill traffic, s_load = kernarg rematerialisation, LDS ops).

    hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 --cuda-device-only -S \
        csrc/hip_tb3.hip -o /tmp/tb3.s
    python tools/kernel_resources.py /tmp/tb3.s k_tb3
"""
import collections
import re
import subprocess
import sys


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names),
                             capture_output=True, text=True, check=True).stdout.split("\n")
        return out[:len(names)]
    except Exception:
        return names


def kernels(text):
    """yield (name, body, metadata dict) per kernel"""
    meta = {}
    for blk in re.finditer(r"- \.agpr_count:.*?\.name:\s+(\S+)(.*?)(?=\n  - \.agpr|\namdhsa|\s*\.end_amdgpu_metadata)", text, re.S):
        name = blk.group(1)
        d = {}
        for k in ("agpr_count", "vgpr_count", "sgpr_count", "sgpr_spill_count", "vgpr_spill_count",
                  "group_segment_fixed_size", "private_segment_fixed_size"):
            m = re.search(r"\." + k + r":\s+(\d+)", blk.group(0))
            d[k] = int(m.group(1)) if m else -1
        meta[name] = d
    for name, d in meta.items():
        start = text.find("\n" + name + ":")
        end = text.find(".Lfunc_end", start)
        yield name, text[start:end] if start >= 0 else "", d


def summary(path, filt):
    text = open(path).read()
    rows = []
    for name, body, d in kernels(text):
        if filt not in name:
            continue
        c = collections.Counter()
        for line in body.split("\n"):
            t = line.strip()
            if not t or t[0] in ";." or t.endswith(":"):
                continue
            c[t.split()[0]] += 1
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        pk = sum(v for k, v in c.items() if k.startswith("v_pk_"))
        lds = sum(v for k, v in c.items() if k.startswith("ds_"))
        sload = sum(v for k, v in c.items() if k.startswith("s_load"))
        rows.append((name, d, valu, pk, c["v_readlane_b32"], c["v_writelane_b32"], sload, lds))
    dn = demangle([r[0] for r in rows])
    print("%-6s %-6s %-6s %-7s %-7s %-6s %-6s %-6s %-5s %-5s %-6s %-5s  kernel" %
          ("vgpr", "agpr", "sgpr", "sspill", "vspill", "lds", "scr", "valu", "v_pk", "rdln", "wrln", "sload"))
    for (name, d, valu, pk, rl, wl, sl, lds), dname in zip(rows, dn):
        print("%-6d %-6d %-6d %-7d %-7d %-6d %-6d %-6d %-5d %-5d %-6d %-5d  %s" %
              (d["vgpr_count"], d["agpr_count"], d["sgpr_count"], d["sgpr_spill_count"], d["vgpr_spill_count"],
               d["group_segment_fixed_size"], d["private_segment_fixed_size"], valu, pk, rl, wl, sl,
               dname.replace("wave3d::(anonymous namespace)::", "")))


if __name__ == "__main__":
    summary(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
