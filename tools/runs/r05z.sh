# Round 5 (closing tree): smoke and the default bench (python bench.py, as
# the driver runs it).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r05z_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r05z_bench.json 2> gpurun_out/r05z_bench.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05z_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["avg_kernel_ms"], d["roofline"]["event_stride"], {k: d[k]["ms_per_step"] for k in d if isinstance(d[k], dict) and "ms_per_step" in d[k]})
PY
