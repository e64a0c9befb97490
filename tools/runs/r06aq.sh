# Round 6: form 12's 64-row tiles with every weight strip requested a phase
# ahead (TFL_PRE12=1, the 16-row tiles' schedule) against each strip loaded in
# the phase that uses it (build_old: -DTFL_PRE12=0) - decoder kernel stats at
# B=128 T=2600, alternated twice; tile tests on the new build.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_range.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06aq_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06aq_tests.log; [ $rc -eq 0 ] || exit $rc
OLD=m2-tts_amd/csrc/build_old/libm2tts_hip_old.so
NEW=m2-tts_amd/src/m2amd/libm2tts_hip.so
for i in 1 2; do
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  M2TTS_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06aq_${v}_$i -o run -- python3 tools/probe/dec_time.py 128 2600 10 > gpurun_out/r06aq_${v}_$i.log 2>&1 || exit 1
  rm -f gpurun_out/r06aq_${v}_$i/run_kernel_trace.csv
  python3 - gpurun_out/r06aq_${v}_$i $v <<'PY' >> gpurun_out/r06aq_ab.txt
import csv, sys
for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_stats.csv")):
    if "layer_kernel" in r["Name"] or "first_kernel" in r["Name"]:
        print(sys.argv[2], r["Name"].split("(")[0][5:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
done
cat gpurun_out/r06aq_ab.txt
