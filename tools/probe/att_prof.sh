#!/bin/bash
# rocprofv3 kernel stats of the pipeline workload: the default library, the
# exact-f32 attention (M2_ATT_F32=1) and any variant libraries given by name
# (m2-tts_amd/csrc/build_v<name>/libm2tts_hip_v<name>.so).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python3 bench.py --workload pipeline --no-cpu-baseline --no-pipeline-extra --steps 100 --warmup 100"
timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/att_split -o run -- $B > gpurun_out/att_split.log 2>&1 || exit 1
M2_ATT_F32=1 timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/att_f32 -o run -- $B > gpurun_out/att_f32.log 2>&1 || exit 1
for n in "$@"; do
  M2TTS_HIP_LIB=m2-tts_amd/csrc/build_v$n/libm2tts_hip_v$n.so timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/att_$n -o run -- $B > gpurun_out/att_$n.log 2>&1 || exit 1
done
