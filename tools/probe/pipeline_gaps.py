#!/usr/bin/env python3
"""Idle gaps between consecutive kernel dispatches of the pipeline bench
(rocprofv3 --kernel-trace csv): median gap before each kernel of a step.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps -o run -- \
        python3 bench.py --workload pipeline --steps 50 --warmup 50 --no-cpu-baseline --no-pipeline-extra
    python tools/probe/pipeline_gaps.py gpurun_out/gaps
"""
import csv
import glob
import statistics
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"][:60] for r in rows]
st = [int(r["Start_Timestamp"]) for r in rows]
en = [int(r["End_Timestamp"]) for r in rows]
# a step starts at the embedding kernel
starts = [i for i, n in enumerate(names) if "embed_pe_kernel" in n]
per = {}
steps = []
for a, b in zip(starts[len(starts) // 2:-1], starts[len(starts) // 2 + 1:]):
    steps.append((st[b] - st[a]) / 1e3)
    for k, i in enumerate(range(a, b)):
        gap = (st[i] - en[i - 1]) / 1e3 if i > 0 else 0.0
        per.setdefault(k, (names[i], []))[1].append((gap, (en[i] - st[i]) / 1e3))
print(f"steps {len(steps)}, median step {statistics.median(steps):.1f} us")
tg = 0.0
for k, (n, v) in sorted(per.items()):
    g = statistics.median(x[0] for x in v)
    d = statistics.median(x[1] for x in v)
    tg += g
    print(f"{k:3d} gap {g:7.2f}  dur {d:7.2f}  {n}")
print(f"sum of median gaps {tg:.1f} us")
