# Round 5: phase stamps of the one-launch transformer layer at the configs[3]
# B=8 share (encoder 8x100, decoder 8x500) on the round-5 default forms.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so timeout -k 10 120 python -u tools/probe/tfl_stamps.py s2 enc8x100 8x500 > gpurun_out/r05ad_stamps.txt 2>&1
rc=$?; cat gpurun_out/r05ad_stamps.txt; [ $rc -eq 0 ] || exit $rc
