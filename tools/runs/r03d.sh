# Round 3: L2 read bandwidth per CU, stamps of the one-launch layers after the
# wait fix, the general-component tests, traces, bench.
set -u
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probe/l2bw.bin 458752 256 512 > gpurun_out/r03d_l2bw.txt 2>&1 &&
timeout -k 10 60 ./tools/probe/l2bw.bin 229376 256 512 >> gpurun_out/r03d_l2bw.txt 2>&1 &&
timeout -k 10 60 ./tools/probe/l2bw.bin 458752 256 256 >> gpurun_out/r03d_l2bw.txt 2>&1 &&
timeout -k 10 60 ./tools/probe/l2bw.bin 458752 512 512 >> gpurun_out/r03d_l2bw.txt 2>&1
rc=$?; cat gpurun_out/r03d_l2bw.txt; [ $rc -eq 0 ] || exit $rc
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so timeout -k 10 120 python -u tools/probe/tfl_stamps.py s2 8x500 64x500 > gpurun_out/r03d_stamps.txt 2>&1
rc=$?; cat gpurun_out/r03d_stamps.txt | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_components_general.py tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03d_comp.log 2>&1
rc=$?; tail -5 gpurun_out/r03d_comp.log; [ $rc -eq 0 ] || exit $rc
bash tools/probe/s2_small_trace.sh
