# Round 6 (start): GPU suite, smoke and the driver-form bench on the round-5 tree.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06a_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/r06a_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/r06a_gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06a_smoke.log 2>&1 || { tail -n 20 gpurun_out/r06a_smoke.log; exit 1; }
tail -n 1 gpurun_out/r06a_smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06a_bench_driver.json 2> gpurun_out/r06a_bench_driver.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06a_bench_driver.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["cpu_baseline"]["value"], {k: d[k]["ms_per_step"] for k in d if isinstance(d[k], dict) and "ms_per_step" in d[k]})
PY
