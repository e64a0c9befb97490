#!/usr/bin/env python3
"""Attention kernel rows of tools/probe/att_prof.sh outputs: python tools/probe/att_table.py split f32 ..."""
import csv
import sys
for n in sys.argv[1:]:
    for r in csv.DictReader(open(f"gpurun_out/att_{n}/run_kernel_stats.csv")):
        if "attention" in r["Name"]:
            print(f"{n:8s} {r['Name'][:40]:40s} {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:6.2f} us  "
                  f"min {float(r['MinNs'])/1e3:6.2f}  max {float(r['MaxNs'])/1e3:6.2f}")
