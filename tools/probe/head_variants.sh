#!/bin/bash
# Head tiling variants (libraries built with different X3_* macros under
# m2-tts_amd/csrc/build_v<name>/): rocprofv3 kernel stats per variant.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in "$@"; do
  M2TTS_HIP_LIB=m2-tts_amd/csrc/build_v$n/libm2tts_hip_v$n.so timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/var_$n -o run -- python3 bench.py --no-cpu-baseline --no-pipeline-extra --steps 300 --warmup 300 > gpurun_out/var_$n.log 2>&1 || exit 1
done
