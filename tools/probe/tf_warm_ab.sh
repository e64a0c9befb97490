# L2 warm-up of the 8-wave post_attn layers: parity, B=8 kernel trace, and a
# bench A/B against a -DTF_WARM=0 build (make OBJDIR=build_nw ...).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
NW=m2-tts_amd/csrc/build_nw/libm2tts_hip_nw.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tfwarm_tests.log 2>&1 || { tail -n 20 gpurun_out/tfwarm_tests.log; exit 1; }
tail -n 1 gpurun_out/tfwarm_tests.log
for v in warm nowarm; do
  L=""; [ $v = nowarm ] && L=$NW
  M2TTS_HIP_LIB=${L:-m2-tts_amd/src/m2amd/libm2tts_hip.so} timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tfwarm_$v -o run -- python3 tools/probe/s2_small_trace.py 8 > gpurun_out/tfwarm_$v.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize gpurun_out/tfwarm_$v/run_kernel_trace.csv > gpurun_out/tfwarm_$v.txt || exit 1
  rm -f gpurun_out/tfwarm_$v/run_kernel_trace.csv
done
for i in 1 2; do
  for v in warm nowarm; do
    L=""; [ $v = nowarm ] && L=$NW
    M2TTS_HIP_LIB=${L:-m2-tts_amd/src/m2amd/libm2tts_hip.so} timeout -k 10 200 python bench.py --workload pipeline --no-extras --no-cpu-baseline --steps 300 --warmup 20 > gpurun_out/tfwarm_pipe_${v}_$i.json 2>/dev/null || exit 1
  done
done
