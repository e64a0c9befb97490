# Round 4, after the 4-wave first launch: the full GPU suite, smoke and the
# default bench on the final library, and configs[4]'s kernel trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ai_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04ai_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04ai_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/r04ai_smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/r04ai_bench.json 2> gpurun_out/r04ai_bench.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r04ai_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], {k: d[k]["ms_per_step"] for k in d if isinstance(d[k], dict) and "ms_per_step" in d[k]})
PY
d=gpurun_out/r04ai_tr_128_one_520
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $d.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 3 > $d.txt || exit 1
rm -f $d/run_kernel_trace.csv
head -3 $d.txt
