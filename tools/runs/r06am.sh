# Round 6: phase stamps of the key-quarter layer (-DTFL_STAMPS build) - the
# decoder's last layer at B=128 T=2600 and B=16 T=2600: attention loop, merge,
# out-proj, LN2, FFN1, FFN2.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so timeout -k 10 300 python -u tools/probe/tfl_stamps.py s2 128x2600 16x2600 > gpurun_out/r06am_stamps.txt 2>&1 || { tail -20 gpurun_out/r06am_stamps.txt; exit 1; }
cat gpurun_out/r06am_stamps.txt
