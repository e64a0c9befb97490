# Round 5: stage2 mid kernel B-fragment prefetch (X3S2_MBP=1 both planes,
# =2 hi only; tools/probe/libm2tts_mbp{1,2}.so) against the in-tree library
# (MBP 0): parity with each, then kernel stats of the stage2 vocoder shapes,
# alternated twice.
set -u
tag=r05l
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in mbp1 mbp2; do
  M2TTS_HIP_LIB=tools/probe/libm2tts_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_head_comp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_${v}_tests.log 2>&1 || { tail -n 20 gpurun_out/${tag}_${v}_tests.log; exit 1; }
  tail -n 1 gpurun_out/${tag}_${v}_tests.log
done
for i in 1 2; do
for v in base mbp1 mbp2; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v != base ] && L=tools/probe/libm2tts_$v.so
  for sh in 8x500 16x2600; do
    M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_${sh}_${v}_$i -o run -- \
        python3 bench.py --workload s2_vocoder --s2-shape $sh --steps 30 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/${tag}_${sh}_${v}_$i.json 2>/dev/null || exit 1
    rm -f gpurun_out/${tag}_${sh}_${v}_$i/run_kernel_trace.csv
  done
done
done
