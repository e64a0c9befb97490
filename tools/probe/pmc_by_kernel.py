#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection.csv rows per kernel name (median per
dispatch): python tools/probe/pmc_by_kernel.py DIR/run_counter_collection.csv [name-filter]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    per = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if filt and filt not in name:
            continue
        per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in per.items():
        print(name[:90])
        for c, v in sorted(cs.items()):
            v.sort()
            print(f"   {c:28s} median {v[len(v) // 2]:14.0f}  (n {len(v)})")


if __name__ == "__main__":
    main()
