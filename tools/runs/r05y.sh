# Round 5: the length regulator's count as one wave per utterance: the GPU
# suite, then kernel stats of the stage1 pipeline against the previous
# library (m2-tts_amd/csrc/build_old), alternated.
set -u
tag=r05y
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
OLD=m2-tts_amd/csrc/build_old/libm2tts_hip_old.so
NEW=m2-tts_amd/src/m2amd/libm2tts_hip.so
for i in 1 2; do
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_${v}_$i -o run -- \
      python3 bench.py --workload pipeline --steps 100 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/${tag}_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/${tag}_${v}_$i/run_kernel_trace.csv
done
done
