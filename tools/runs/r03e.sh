# Round 3: the per-XCD work queue of the one-launch layers: stamps, tests, traces.
set -u
mkdir -p gpurun_out
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so timeout -k 10 120 python -u tools/probe/tfl_stamps.py s2 8x500 64x500 enc8x100 > gpurun_out/r03e_stamps.txt 2>&1
rc=$?; cat gpurun_out/r03e_stamps.txt | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_components_general.py tests/test_gpu_tf_layer.py tests/test_gpu_sharding_streaming.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03e_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r03e_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/probe/s2_small_trace.sh && cat gpurun_out/s2t_b8.txt gpurun_out/s2t_b64.txt
