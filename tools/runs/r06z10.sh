# M2_KB8 (the exact-f32 kernels' weight double buffer at 8 k-steps = 2 KiB per
# wave in flight) as a separate library build, processes alternated.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r06z10_kb8.txt
: > $O
for i in 1 2 3; do
  echo "== default (KB 4)" >> $O
  timeout -k 10 100 python3 -u tools/probe/voc_env_ab.py M2_F32_MT 2 1 s1 32 500 4 40 2>/dev/null | tail -1 >> $O || exit 1
  echo "== KB8" >> $O
  M2TTS_HIP_LIB=$PWD/m2-tts_amd/csrc/build_kb8/libm2tts_kb8.so timeout -k 10 100 python3 -u tools/probe/voc_env_ab.py M2_F32_MT 2 1 s1 32 500 4 40 2>/dev/null | tail -1 >> $O || exit 1
done
cat $O
