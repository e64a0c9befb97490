# Round 4, first record: the switch table, the one-launch guarded redo, the
# pipeline lanes' own handles, the RCCL test (skips on one GPU); full GPU
# suite, smoke, default bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04a_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04a_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04a_smoke.log 2>&1 || exit 1
tail -3 gpurun_out/r04a_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r04a_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], {k: d[k]["ms_per_step"] for k in ("pipeline", "vocoder_report_policy", "s2_vocoder_b8_t500", "s2_vocoder_b16_t2600", "s2_b64_sharded", "s2_b64_sharded_2inflight", "s2_b8_per_gpu_share", "s2_b8_per_gpu_share_2inflight", "s2_longform_sharded")}, d.get("cpu_baseline", {}).get("value"))
print({k: d[k].get("parity") for k in ("s2_b64_sharded", "s2_b64_sharded_2inflight", "s2_b8_per_gpu_share", "s2_longform_sharded")})
print(d["vocoder_report_policy"])
PY
