# Round 6: N=4 rehearsal of the sharded lines with gloo, four ranks sharing
# the one GPU (the HIP phases, device-T flow and ShardedPipeline at world 4;
# gloo stages the collectives through the host, so times are not RCCL's).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --gpus 4 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06ab_bench_n4_gloo.json 2> gpurun_out/r06ab_bench_n4_gloo.err || { tail -n 30 gpurun_out/r06ab_bench_n4_gloo.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06ab_bench_n4_gloo.json").read().strip().splitlines()[-1])
print(d["n_gpus"], d["value"], d["ms_per_step"])
print({k: (d[k]["ms_per_step"], d[k].get("parity")) for k in d if isinstance(d[k], dict) and "parity" in d[k]})
PY
