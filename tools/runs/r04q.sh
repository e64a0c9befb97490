# Round 4: the default bench with the like-for-like report-policy line.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > gpurun_out/r04q_bench.json 2> gpurun_out/r04q_bench.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r04q_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["traffic"])
print(json.dumps(d["vocoder_report_policy"]))
PY
