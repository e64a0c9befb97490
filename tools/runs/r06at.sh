# Round 6: phase stamps of the 16-row-tile layers at configs[3]'s share
# (stage2 B=8 T=500 decoder, S=100 encoder).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so timeout -k 10 300 python -u tools/probe/tfl_stamps.py s2 8x500 enc8x100 > gpurun_out/r06at_stamps.txt 2>&1 || { tail -20 gpurun_out/r06at_stamps.txt; exit 1; }
cat gpurun_out/r06at_stamps.txt
