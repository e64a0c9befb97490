#!/bin/bash
# Stage2 x3 tiling variants (libraries built with X3S2_* macros under
# m2-tts_amd/csrc/build_v<name>/): s2 parity tests + s2 vocoder bench lines.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then lib=m2-tts_amd/src/m2amd/libm2tts_hip.so; else lib=m2-tts_amd/csrc/build_v$v/libm2tts_hip_v$v.so; fi
  M2TTS_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharding_streaming.py -m gpu -x -q -k "s2" --timeout 120 --timeout-method thread > gpurun_out/s2t_${v}_tests.log 2>&1 || { tail -5 gpurun_out/s2t_${v}_tests.log; exit 1; }
  for sh in 8x500 16x2600 64x500; do
    M2TTS_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --workload s2_vocoder --s2-shape $sh --no-extras --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/s2t_${v}_${sh}.json 2> gpurun_out/s2t_${v}_${sh}.err || exit 1
  done
done
