# Round 6: lean split-stream ShardedPipeline - pipeline / sharding / stress tests,
# the host-cost probe, and the N=2 gloo rehearsal.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_T.py tests/test_gpu_sharding_streaming.py tests/test_gpu_stress.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06i_tests.log 2>&1 || { tail -n 30 gpurun_out/r06i_tests.log; exit 1; }
tail -n 1 gpurun_out/r06i_tests.log
timeout -k 10 300 python3 -u tools/probe/pipe_host.py 200 > gpurun_out/r06i_pipe_host.txt 2>&1 || { tail -n 30 gpurun_out/r06i_pipe_host.txt; exit 1; }
cat gpurun_out/r06i_pipe_host.txt
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06i_bench_n2.json 2> gpurun_out/r06i_bench_n2.err || { tail -n 20 gpurun_out/r06i_bench_n2.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06i_bench_n2.json").read().strip().splitlines()[-1])
print({k: (d[k]["ms_per_step"], d[k].get("parity", {}).get("bitwise_equal")) for k in d if isinstance(d[k], dict) and "parity" in d[k]})
PY
