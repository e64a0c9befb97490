# Round 5: B-fragment reads one k-block ahead in mma_x3 (X3_BPIPE=1 build in
# tools/probe/libm2tts_bpipe.so) against the in-tree library: vocoder parity
# with the variant, then kernel stats of the stage1 headline and the stage2
# vocoder shapes for both, alternated twice.
set -u
tag=r05g
export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=tools/probe/libm2tts_bpipe.so
OLD=m2-tts_amd/src/m2amd/libm2tts_hip.so
M2TTS_HIP_LIB=$NEW timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_head_comp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 20 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
for i in 1 2; do
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_s1_${v}_$i -o run -- \
      python3 bench.py --workload vocoder --steps 100 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/${tag}_s1_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/${tag}_s1_${v}_$i/run_kernel_trace.csv
  for sh in 8x500 16x2600; do
    M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_s2_${sh}_${v}_$i -o run -- \
        python3 bench.py --workload s2_vocoder --s2-shape $sh --steps 30 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/${tag}_s2_${sh}_${v}_$i.json 2>/dev/null || exit 1
    rm -f gpurun_out/${tag}_s2_${sh}_${v}_$i/run_kernel_trace.csv
  done
done
done
