# Round 3: two global batches in flight (ShardedPipeline): tests, bench, traces.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_T.py tests/test_gpu_sharding_streaming.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03p_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r03p_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r03p_bench.json 2> gpurun_out/r03p_bench.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r03p_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], {k: d[k]["ms_per_step"] for k in ("pipeline", "s2_vocoder_b8_t500", "s2_b64_sharded", "s2_b64_sharded_2inflight", "s2_b8_per_gpu_share", "s2_b8_per_gpu_share_2inflight", "s2_longform_sharded")})
PY
