# Round 6 re-entry closing record on the two-phase exact-f32 tail tree (the GPU
# suite ran as r06z4 on the same kernels): smoke, the default bench, the
# headline kernel stats + PMC passes, the N=2 gloo rehearsal.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06z5_smoke.log 2>&1 || { tail -n 20 gpurun_out/r06z5_smoke.log; exit 1; }
tail -n 1 gpurun_out/r06z5_smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/r06z5_bench.json 2> gpurun_out/r06z5_bench.err || { tail -n 20 gpurun_out/r06z5_bench.err; exit 1; }
grep "ms/step" gpurun_out/r06z5_bench.err
bash tools/profile_gpu.sh r06z5 || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_r06z5 --traffic gpurun_out/r06z5_traffic.json > gpurun_out/r06z5_pmc.txt || exit 1
python3 tools/prof_summary.py gpurun_out/prof_r06z5 > gpurun_out/r06z5_prof.txt 2>&1 || true
cat gpurun_out/r06z5_traffic.json
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06z5_bench_n2.json 2> gpurun_out/r06z5_bench_n2.err || { tail -n 20 gpurun_out/r06z5_bench_n2.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06z5_bench_n2.json").read().strip().splitlines()[-1])
print({k: (d[k]["ms_per_step"], d[k].get("parity", {}).get("bitwise_equal")) for k in d if isinstance(d[k], dict) and "parity" in d[k]})
PY
