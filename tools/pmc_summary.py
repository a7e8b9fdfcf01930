#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output (one dir per pass) per kernel: mean per dispatch."""
import collections
import csv
import glob
import sys


def summarise(root, match):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    durs = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{root}/pmc_*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if match not in r["Kernel_Name"]:
                continue
            per[(f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for f in sorted(glob.glob(f"{root}/pmc_*/run_kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            if match in r["Kernel_Name"]:
                durs[f].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = collections.defaultdict(list)
    for cs in per.values():
        for c, v in cs.items():
            tot[c].append(v)
    out = {c: sum(v) / len(v) for c, v in tot.items()}
    alld = [d for v in durs.values() for d in v]
    out["duration_ns_median"] = sorted(alld)[len(alld) // 2] if alld else 0
    return out


if __name__ == "__main__":
    root, match = sys.argv[1], sys.argv[2]
    s = summarise(root, match)
    for k in sorted(s):
        print(f"{k:26s} {s[k]:18.1f}")
    if "SQ_WAVE_CYCLES" in s:
        w = s["SQ_WAVE_CYCLES"]
        print(f"{'frac WAIT_ANY':26s} {s['SQ_WAIT_ANY']/w:18.3f}")
        print(f"{'frac WAIT_INST_ANY':26s} {s['SQ_WAIT_INST_ANY']/w:18.3f}")
        print(f"{'frac ACTIVE_INST_ANY':26s} {s['SQ_ACTIVE_INST_ANY']/w:18.3f}")
