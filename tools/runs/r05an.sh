# Round 5 (closing): the driver's default bench command on the final tree.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > gpurun_out/r05an_bench.json 2> gpurun_out/r05an_bench.err || { tail -n 20 gpurun_out/r05an_bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05an_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["avg_kernel_ms"], d["cpu_baseline"]["value"], d["cpu_baseline"]["spread"])
PY
