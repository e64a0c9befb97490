# Round 5 (later tree): the full GPU suite, smoke and the default bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05m_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05m_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05m_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r05m_smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/r05m_bench.json 2> gpurun_out/r05m_bench.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05m_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], {k: d[k]["ms_per_step"] for k in d if isinstance(d[k], dict) and "ms_per_step" in d[k]})
PY
