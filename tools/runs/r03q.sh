# Round 3: long-form decoder layer at B=128 T=2600 (configs[4]), layer phase stamps at B=8 (encoder / decoder).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so timeout -k 10 120 python -u tools/probe/tfl_stamps.py s2 enc8x100 8x500 128x2600 > gpurun_out/r03q_stamps.txt 2>&1
rc=$?; cat gpurun_out/r03q_stamps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2t_lf128 -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > gpurun_out/s2t_lf128.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/s2t_lf128/run_kernel_trace.csv 10 > gpurun_out/s2t_lf128.txt || exit 1
rm -f gpurun_out/s2t_lf128/run_kernel_trace.csv; cat gpurun_out/s2t_lf128.txt
