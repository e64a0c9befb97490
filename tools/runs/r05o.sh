# Round 5: kernel time line of the headline vocoder (start / end of every
# kernel): the gaps between the three launches of a call and between calls.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG:-r05o} -o run -- \
    python3 bench.py --workload vocoder --steps 50 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/${TAG:-r05o}.json 2>/dev/null || exit 1
python3 - > gpurun_out/${TAG:-r05o}_gaps.txt <<'PY'
import csv
rows = sorted(csv.DictReader(open("gpurun_out/" + __import__("os").environ.get("TAG", "r05o") + "/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if any(k in r["Kernel_Name"] for k in ("x3_head", "midp", "tailp"))][-150:]
import statistics as st
dur = {}
gap = {}
for a, b in zip(rows, rows[1:]):
    na = a["Kernel_Name"].split("(")[0][-40:]; nb = b["Kernel_Name"].split("(")[0][-40:]
    gap.setdefault((na, nb), []).append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
for r in rows:
    n = r["Kernel_Name"].split("(")[0][-40:]
    dur.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in dur.items(): print("dur", k, round(st.median(v), 2))
for k, v in gap.items(): print("gap", k, round(st.median(v), 2), "min", round(min(v), 2))
PY
cat gpurun_out/${TAG:-r05o}_gaps.txt; rm -f gpurun_out/${TAG:-r05o}/run_kernel_trace.csv
