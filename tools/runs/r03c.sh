# Round 3: phase stamps of the one-launch layers, the general-component tests,
# the B=8 / B=64 traces and the driver-form bench.
set -u
mkdir -p gpurun_out
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so timeout -k 10 120 python -u tools/probe/tfl_stamps.py s2 8x500 enc8x100 64x500 > gpurun_out/r03c_stamps.txt 2>&1
rc=$?; cat gpurun_out/r03c_stamps.txt | tail -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_components_general.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03c_comp.log 2>&1
rc=$?; tail -5 gpurun_out/r03c_comp.log; [ $rc -eq 0 ] || exit $rc
bash tools/probe/s2_small_trace.sh &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03c_bench_driver.json 2> gpurun_out/r03c_bench_driver.err
