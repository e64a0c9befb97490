# Round 3 re-entry check on the rebuilt tree: full GPU suite, smoke, default bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03y_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r03y_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03y_smoke.log 2>&1 || exit 1
cat gpurun_out/r03y_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03y_bench.json 2> gpurun_out/r03y_bench.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r03y_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], {k: d[k]["ms_per_step"] for k in ("pipeline", "s2_vocoder_b8_t500", "s2_vocoder_b16_t2600", "s2_b64_sharded", "s2_b8_per_gpu_share", "s2_b8_per_gpu_share_2inflight", "s2_longform_sharded") if k in d})
PY
