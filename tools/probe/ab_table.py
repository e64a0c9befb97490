#!/usr/bin/env python3
"""Kernel averages (us) per arm of tools/probe/lib_ab.sh: ab_table.py <tag> [filter...]"""
import csv
import glob
import json
import sys

tag, filt = sys.argv[1], sys.argv[2:]
for d in sorted(glob.glob(f"gpurun_out/{tag}_*_[12]")):
    arm = d.split("/")[-1]
    try:
        ms = json.load(open(d + ".json"))["ms_per_step"]
    except Exception:
        ms = None
    out = []
    for r in csv.DictReader(open(d + "/run_kernel_stats.csv")):
        n = r["Name"].split("(")[0].replace("void ", "")
        if not filt or any(f in n for f in filt):
            out.append(f"{n[-45:]}={float(r['AverageNs']) / 1e3:.2f}")
    print(arm, "ms/step", ms, " ".join(out))
