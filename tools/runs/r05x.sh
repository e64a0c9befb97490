# Round 5 (closing): driver-form bench, the headline kernel trace + PMC passes.

set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05x_bench_driver.json 2> gpurun_out/r05x_bench_driver.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05x_bench_driver.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], {k: d[k]["ms_per_step"] for k in d if isinstance(d[k], dict) and "ms_per_step" in d[k]})
PY
bash tools/profile_gpu.sh r05x || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_r05x --traffic gpurun_out/r05x_traffic.json > gpurun_out/r05x_pmc.txt || exit 1
python3 tools/prof_summary.py gpurun_out/prof_r05x > gpurun_out/r05x_prof.txt 2>&1 || true
cat gpurun_out/r05x_traffic.json
