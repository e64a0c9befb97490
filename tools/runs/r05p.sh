# Round 5: kernel timing by dispatch timestamps (m2_launch): GPU suite, the
# kernel time line with events on every call, then the default bench.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05p_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05p_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
TAG=r05p bash tools/runs/r05o.sh || exit 1
timeout -k 10 500 python -u bench.py > gpurun_out/r05p_bench.json 2> gpurun_out/r05p_bench.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05p_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"], {k: d[k]["ms_per_step"] for k in d if isinstance(d[k], dict) and "ms_per_step" in d[k]})
PY
