# Round 4: is the LDS-DMA wave-specialised attention (M2_TFL_QS2=9) bound by
# its one-step DMA lead?  Diagnostic builds: producers not waiting for their
# DMAs before the step barrier (TFL_DIAG=32), or issuing none after step 0
# (64); decoder alone at B=128 T=2600.  Then the untied-region + DMA form (10)
# against 9 in-process.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in 0 32 64; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $d != 0 ] && L=m2-tts_amd/csrc/build_diag/libm2tts_hip_d$d.so
  M2TTS_HIP_LIB=$L M2_TFL_QS2=9 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04o_d$d -o run -- python3 tools/probe/dec_time.py 128 2600 6 > gpurun_out/r04o_d$d.log 2>&1 || exit 1
  rm -f gpurun_out/r04o_d$d/run_kernel_trace.csv
  python3 - gpurun_out/r04o_d$d/run_kernel_stats.csv "diag $d $(grep decoder gpurun_out/r04o_d$d.log)" <<'PY'
import csv, sys
print(sys.argv[2], " | ".join(f'{r["Name"].split("(")[0].replace("void m2::tfl::", "")} {float(r["AverageNs"]) / 1e3:.1f}us' for r in csv.DictReader(open(sys.argv[1])) if "layer_kernel" in r["Name"]))
PY
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread -k "4q10 or 4q9" > gpurun_out/r04o_tf_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04o_tf_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 9,10 s2 128 520 4 2 > gpurun_out/r04o_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r04o_ab_lf.txt
