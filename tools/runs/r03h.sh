# Round 3: launch gaps of the stage2 B=8 step, two-phase (front/back) vs one call.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for mode in two one; do
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2g_$mode -o run -- python3 tools/probe/s2_small_trace.py 8 $mode > gpurun_out/s2g_$mode.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/s2g_$mode/run_kernel_trace.csv > gpurun_out/s2g_$mode.txt || exit 1
rm -f gpurun_out/s2g_$mode/run_kernel_trace.csv
cat gpurun_out/s2g_$mode.txt
done
timeout -k 10 60 tools/probe/l2bw.bin 458752 > gpurun_out/l2bw_448k.txt 2>&1 || exit 1
timeout -k 10 60 tools/probe/l2bw.bin 1572864 > gpurun_out/l2bw_1536k.txt 2>&1 || exit 1
cat gpurun_out/l2bw_448k.txt gpurun_out/l2bw_1536k.txt
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so timeout -k 10 120 python -u tools/probe/tfl_stamps.py s2 8x500 64x500 > gpurun_out/r03h_stamps.txt 2>&1 || exit 1
cat gpurun_out/r03h_stamps.txt
