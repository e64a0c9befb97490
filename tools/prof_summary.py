#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (results .db or
kernel_stats.csv) into a per-kernel table: calls, total/avg/min/max us, %.

    python tools/prof_summary.py gpurun_out/prof1 [--out profiles/r01_x.csv]
"""
import argparse
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    db = sqlite3.connect(path)
    rows = db.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                      "from kernels group by name order by sum(duration) desc").fetchall()
    return [(n, c, t / 1e3, a / 1e3, mn / 1e3, mx / 1e3) for n, c, t, a, mn, mx in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3,
                        float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    dbs = glob.glob(os.path.join(a.dir, "**", "*results.db"), recursive=True)
    csvs = glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True)
    rows = from_csv(csvs[0]) if csvs else from_db(dbs[0])
    tot = sum(r[2] for r in rows) or 1.0
    w = csv.writer(open(a.out, "w", newline="")) if a.out else csv.writer(sys.stdout)
    w.writerow(["kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "pct"])
    for n, c, t, av, mn, mx in rows:
        w.writerow([n[:160], c, f"{t:.1f}", f"{av:.2f}", f"{mn:.2f}", f"{mx:.2f}", f"{100 * t / tot:.1f}"])


if __name__ == "__main__":
    main()
