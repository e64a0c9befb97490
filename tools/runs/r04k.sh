# Round 4, second record: the full GPU suite, smoke and default bench on the
# ping-pong attention / plane swizzle / XCD-aware head build; headline A/B of
# the XCD-aware head windows against the plain order (X3_HEAD_XCD=0 build).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04k_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04k_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04k_smoke.log 2>&1 || exit 1
tail -3 gpurun_out/r04k_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r04k_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], {k: d[k]["ms_per_step"] for k in ("pipeline", "vocoder_report_policy", "s2_vocoder_b8_t500", "s2_vocoder_b16_t2600", "s2_b64_sharded", "s2_b64_sharded_2inflight", "s2_b8_per_gpu_share", "s2_b8_per_gpu_share_2inflight", "s2_longform_sharded")}, d.get("cpu_baseline", {}).get("value"))
print({k: d[k].get("parity") for k in ("s2_b64_sharded", "s2_b64_sharded_2inflight", "s2_b8_per_gpu_share", "s2_longform_sharded")})
PY
NOX=m2-tts_amd/csrc/build_ab/libm2tts_hip_noxcd.so
for i in 1 2 3; do for v in xcd plain; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v = plain ] && L=$NOX
  M2TTS_HIP_LIB=$L timeout -k 10 200 python3 bench.py --steps 300 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/r04k_hl_${v}$i.json 2>/dev/null || exit 1
  echo "headline $v $i $(python3 -c "import json;print(json.loads(open('gpurun_out/r04k_hl_${v}$i.json').read().strip().splitlines()[-1])['ms_per_step'])")"
done; done
