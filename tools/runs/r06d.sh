# Round 6: ShardedPipeline on split front / back streams - pipeline tests,
# the bench (share lines), an N=2 gloo rehearsal on one GPU.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_T.py tests/test_gpu_sharding_streaming.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06d_tests.log 2>&1 || { tail -n 30 gpurun_out/r06d_tests.log; exit 1; }
tail -n 1 gpurun_out/r06d_tests.log
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r06d_bench.json 2> gpurun_out/r06d_bench.err || { tail -n 20 gpurun_out/r06d_bench.err; exit 1; }
grep "ms/step" gpurun_out/r06d_bench.err
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06d_bench_n2.json 2> gpurun_out/r06d_bench_n2.err || { tail -n 20 gpurun_out/r06d_bench_n2.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06d_bench_n2.json").read().strip().splitlines()[-1])
print({k: (d[k]["ms_per_step"], d[k].get("parity")) for k in d if isinstance(d[k], dict) and "parity" in d[k]})
PY
