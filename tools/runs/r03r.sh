# Round 3 record: full GPU suite, smoke, default bench, driver-form bench, kernel stats (vocoder, pipeline), traces.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03r_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r03r_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03r_smoke.log 2>&1 || exit 1
cat gpurun_out/r03r_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03r_bench.json 2> gpurun_out/r03r_bench.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03r_bench_driver.json 2> gpurun_out/r03r_bench_driver.err || exit 1
python3 - <<'PY'
import json
for f in ("r03r_bench", "r03r_bench_driver"):
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"], {k: d[k]["ms_per_step"] for k in ("pipeline", "s2_vocoder_b8_t500", "s2_vocoder_b16_t2600", "s2_b64_sharded", "s2_b64_sharded_2inflight", "s2_b8_per_gpu_share", "s2_b8_per_gpu_share_2inflight", "s2_longform_sharded")}, d.get("cpu_baseline", {}).get("value"))
PY
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03r_voc -o run -- python3 bench.py --no-cpu-baseline --no-extras --steps 50 --warmup 10 > gpurun_out/r03r_voc.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03r_pipe -o run -- python3 bench.py --workload pipeline --no-cpu-baseline --no-extras --steps 50 --warmup 10 > gpurun_out/r03r_pipe.log 2>&1 || exit 1
rm -f gpurun_out/r03r_voc/run_kernel_trace.csv gpurun_out/r03r_pipe/run_kernel_trace.csv
bash tools/probe/s2_small_trace.sh dev && cat gpurun_out/s2t_dev_b8.txt
