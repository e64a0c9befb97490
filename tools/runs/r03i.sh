# Round 3: the driver-form bench (report policy on the timed lines), and the
# stage2 lines on the three-launch layers (M2_TF_LAYER=0) for comparison.
set -u
mkdir -p gpurun_out
timeout -k 10 420 python -u bench.py > gpurun_out/r03i_bench.json 2> gpurun_out/r03i_bench.err || exit 1
tail -c 600 gpurun_out/r03i_bench.json
M2_TF_LAYER=0 timeout -k 10 300 python -u bench.py --workload s2_b64 --no-cpu-baseline --steps 100 > gpurun_out/r03i_tf0.json 2> gpurun_out/r03i_tf0.err || exit 1
timeout -k 10 300 python -u bench.py --workload s2_b64 --no-cpu-baseline --steps 100 > gpurun_out/r03i_tf1.json 2> gpurun_out/r03i_tf1.err || exit 1
python3 - <<'PY'
import json
for f in ("r03i_bench", "r03i_tf0", "r03i_tf1"):
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    row = {k: (d[k]["ms_per_step"] if isinstance(d.get(k), dict) and "ms_per_step" in d[k] else None)
           for k in ("pipeline", "s2_vocoder_b8_t500", "s2_vocoder_b16_t2600", "s2_b64_sharded", "s2_b8_per_gpu_share",
                     "s2_longform_sharded", "vocoder_default_policy")}
    print(f, d["value"], d["ms_per_step"], row)
PY
