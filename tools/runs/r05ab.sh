# Round 5: stage2 x3 windows at their tile-count limits (build_vall: 8-wave
# head 16 -> 19 frames, 16-wave head 24 -> 27, mid 28 -> 30, small-grid mid
# 32 -> 33; same m-tiles per layer, fewer workgroups) against the in-tree
# library: s2 parity with the variant, bit-identity of the audio across the
# two builds, then kernel stats per shape, alternated twice.
set -u
tag=r05ab
export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=m2-tts_amd/csrc/build_vall/libm2tts_hip_vall.so
OLD=m2-tts_amd/src/m2amd/libm2tts_hip.so
SH="8x500 16x262 16x2600 64x500 128x262"
M2TTS_HIP_LIB=$NEW timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_head_comp.py tests/test_gpu_sharding_streaming.py -m gpu -x -q -k "s2 or head" --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 20 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
M2TTS_HIP_LIB=$NEW timeout -k 10 200 python -u tools/probe/voc_dump.py dump ${tag}_new $SH > gpurun_out/${tag}_dump.log 2>&1 || exit 1
M2TTS_HIP_LIB=$OLD timeout -k 10 200 python -u tools/probe/voc_dump.py dump ${tag}_old $SH >> gpurun_out/${tag}_dump.log 2>&1 || exit 1
python tools/probe/voc_dump.py compare ${tag}_new ${tag}_old $SH > gpurun_out/${tag}_equal.txt 2>&1; cat gpurun_out/${tag}_equal.txt
rm -f gpurun_out/${tag}_*.npy
for i in 1 2; do
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  for sh in $SH; do
    M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_${sh}_${v}_$i -o run -- \
        python3 bench.py --workload s2_vocoder --s2-shape $sh --steps 30 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/${tag}_${sh}_${v}_$i.json 2>/dev/null || exit 1
    rm -f gpurun_out/${tag}_${sh}_${v}_$i/run_kernel_trace.csv
  done
done
done
