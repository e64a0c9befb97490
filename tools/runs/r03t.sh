# Round 3: N=2 rehearsal of the multi-rank bench on one GPU (two ranks, gloo), device-T flow and ShardedPipeline.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03t_n2_gloo.json 2> >(tee gpurun_out/r03t_n2_gloo.err >&2)
rc=$?; tail -5 gpurun_out/r03t_n2_gloo.err; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r03t_n2_gloo.json").read().strip().splitlines()[-1])
print(d["n_gpus"], d["value"], {k: (d[k]["ms_per_step"], d[k]["config"].get("collectives")) for k in ("s2_b64_sharded", "s2_b64_sharded_2inflight", "s2_longform_sharded")})
PY
