# Round 5: hi-only B-fragment prefetch (mma_x3 BP 2) in the stage1 head's
# phase-planar layers and the 16-wave stage2 head of large grids
# (tools/probe/libm2tts_vD.so) against the in-tree library: parity, then
# kernel stats of the headline vocoder and the stage2 long form, alternated.
set -u
tag=r05r
export TMPDIR=/tmp
mkdir -p gpurun_out
M2TTS_HIP_LIB=tools/probe/libm2tts_vD.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_head_comp.py tests/test_gpu_tailp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 20 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
for i in 1 2; do
for v in base vD; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v != base ] && L=tools/probe/libm2tts_$v.so
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_s1_${v}_$i -o run -- \
      python3 bench.py --workload vocoder --steps 100 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/${tag}_s1_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/${tag}_s1_${v}_$i/run_kernel_trace.csv
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_s2_${v}_$i -o run -- \
      python3 bench.py --workload s2_vocoder --s2-shape 16x2600 --steps 30 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/${tag}_s2_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/${tag}_s2_${v}_$i/run_kernel_trace.csv
done
done
