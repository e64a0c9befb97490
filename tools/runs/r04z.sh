# Round 4: the N=2 rehearsal on the final tree (two gloo ranks sharing one
# GPU): the sharded lines' parity against a world-1 inference of the global
# batch.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04z_bench_n2_gloo.json 2> gpurun_out/r04z_bench_n2_gloo.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r04z_bench_n2_gloo.json").read().strip().splitlines()[-1])
print(d["n_gpus"], d["value"], {k: (d[k]["ms_per_step"], d[k].get("parity")) for k in d if isinstance(d[k], dict) and "parity" in d[k]})
PY
