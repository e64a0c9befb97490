# Round 3: hd=48 tail step + 64-row query-split tiles: tf-layer tests, stamps, B=8 / B=64 traces.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_range.py tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03k_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r03k_tests.log; [ $rc -eq 0 ] || exit $rc
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so timeout -k 10 120 python -u tools/probe/tfl_stamps.py s2 8x500 64x500 > gpurun_out/r03k_stamps.txt 2>&1
rc=$?; cat gpurun_out/r03k_stamps.txt; [ $rc -eq 0 ] || exit $rc
bash tools/probe/s2_small_trace.sh && cat gpurun_out/s2t_b8.txt gpurun_out/s2t_b64.txt
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2t_lf16 -o run -- python3 tools/probe/s2_small_trace.py 16 two 520 > gpurun_out/s2t_lf16.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/s2t_lf16/run_kernel_trace.csv 10 > gpurun_out/s2t_lf16.txt || exit 1
rm -f gpurun_out/s2t_lf16/run_kernel_trace.csv
cat gpurun_out/s2t_lf16.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03k_bench.json 2> gpurun_out/r03k_bench.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r03k_bench.json").read().strip().splitlines()[-1])
row = {k: (d[k]["ms_per_step"] if isinstance(d.get(k), dict) and "ms_per_step" in d[k] else None)
       for k in ("pipeline", "s2_vocoder_b8_t500", "s2_vocoder_b16_t2600", "s2_b64_sharded", "s2_b8_per_gpu_share",
                 "s2_longform_sharded", "vocoder_default_policy")}
print(d["value"], d["ms_per_step"], row)
PY
