# Round 5: kernel stats of the stage1 full pipeline (configs[2], B=32 S=100)
# and of configs[3]'s per-GPU share (stage2 B=8 S=100).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05w_pipe -o run -- \
    python3 bench.py --workload pipeline --steps 100 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/r05w_pipe.json 2>/dev/null || exit 1
rm -f gpurun_out/r05w_pipe/run_kernel_trace.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r05w_pipe/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"].split("(")[0][-60:]:60s} calls {r["Calls"]:>6s} avg {float(r["AverageNs"])/1e3:8.2f} us  share {float(r["TotalDurationNs"])/tot:.3f}')
PY
