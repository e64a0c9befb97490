# Round 3: 64-key steps in the query-split attention: tests, stamps, traces, bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03l_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r03l_tests.log; [ $rc -eq 0 ] || exit $rc
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so timeout -k 10 120 python -u tools/probe/tfl_stamps.py s2 64x500 16x2600 > gpurun_out/r03l_stamps.txt 2>&1
rc=$?; cat gpurun_out/r03l_stamps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2t_b64 -o run -- python3 tools/probe/s2_small_trace.py 64 > gpurun_out/s2t_b64.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/s2t_b64/run_kernel_trace.csv > gpurun_out/s2t_b64.txt || exit 1
rm -f gpurun_out/s2t_b64/run_kernel_trace.csv; cat gpurun_out/s2t_b64.txt
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2t_lf16 -o run -- python3 tools/probe/s2_small_trace.py 16 two 520 > gpurun_out/s2t_lf16.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/s2t_lf16/run_kernel_trace.csv 10 > gpurun_out/s2t_lf16.txt || exit 1
rm -f gpurun_out/s2t_lf16/run_kernel_trace.csv; cat gpurun_out/s2t_lf16.txt
