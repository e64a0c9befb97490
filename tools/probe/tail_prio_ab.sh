set -u
mkdir -p gpurun_out
L=m2-tts_amd/csrc/build_vpr/libm2tts_hip_vpr.so
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --no-extras --no-cpu-baseline --steps 400 --warmup 20 > gpurun_out/prio_base_$i.json 2>/dev/null || exit 1
  M2TTS_HIP_LIB=$L timeout -k 10 120 python bench.py --no-extras --no-cpu-baseline --steps 400 --warmup 20 > gpurun_out/prio_alt_$i.json 2>/dev/null || exit 1
done
