set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
L=m2-tts_amd/csrc/build_vpk/libm2tts_hip_vpk.so
for i in 1 2; do
timeout -k 10 120 python tools/probe/att_bench.py --iters 100 > gpurun_out/att_base_$i.json &&
M2TTS_HIP_LIB=$L timeout -k 10 120 python tools/probe/att_bench.py --iters 100 > gpurun_out/att_prio_$i.json || exit 1
done
