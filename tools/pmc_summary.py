#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 PMC passes written by tools/profile_gpu.sh.

    python tools/pmc_summary.py gpurun_out/prof_<tag> [--filter voc_] [--json out.json]

FETCH_SIZE/WRITE_SIZE are in KiB per dispatch (rocprofv3 derived counters);
on gfx950 FETCH_SIZE counts half the bytes of wide streaming reads
(MI355X_MICROARCH.md HBM section), so HBM read bytes = 2 x FETCH_SIZE x 1024.
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(dirpath):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
                cn = r.get("Counter_Name")
                try:
                    v = float(r.get("Counter_Value"))
                except (TypeError, ValueError):
                    continue
                did = r.get("Dispatch_Id")
                per[name][(cn, did)].append(v)
    out = {}
    for name, d in per.items():
        agg = collections.defaultdict(list)
        for (cn, did), vals in d.items():
            agg[cn].append(sum(vals))   # sum over dimensions (XCD/SE instances) per dispatch
        out[name] = {cn: sum(v) / len(v) for cn, v in agg.items()}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--filter", default="")
    ap.add_argument("--json")
    ap.add_argument("--traffic", help="write {kernel short name: HBM bytes per dispatch} (bench.py roofline.traffic)")
    a = ap.parse_args()
    res = {k: v for k, v in load(a.dir).items() if a.filter in k}
    for k, v in sorted(res.items()):
        print(k[:90])
        for cn in sorted(v):
            print(f"   {cn:28s} {v[cn]:.4g}")
        if "FETCH_SIZE" in v or "WRITE_SIZE" in v:
            rd = 2 * v.get("FETCH_SIZE", 0) * 1024
            wr = v.get("WRITE_SIZE", 0) * 1024
            print(f"   -> HBM bytes/dispatch (2xFETCH + WRITE): {rd + wr:.4g}  (read {rd:.4g}, write {wr:.4g})")
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)
    if a.traffic:
        tr = {}
        for k, v in res.items():
            if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
                short = k.split("(")[0].split("<")[0].split("::")[-1].strip()
                tr[short] = round(2 * v["FETCH_SIZE"] * 1024 + v["WRITE_SIZE"] * 1024)
        json.dump(tr, open(a.traffic, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
