# Round 5: run-time strip lengths for the stage1 mid / tail: tests, then the
# headline vocoder (B=32: same strips as before) and B=8 (new strips) against
# the previous library (m2-tts_amd/csrc/build_old), alternated.
set -u
tag=${TAG:-r05u}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tailp.py tests/test_gpu_parity.py tests/test_gpu_range.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 20 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
OLD=m2-tts_amd/csrc/build_old/libm2tts_hip_old.so
NEW=m2-tts_amd/src/m2amd/libm2tts_hip.so
for i in 1 2; do
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  for b in 32 8; do
    M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_b${b}_${v}_$i -o run -- \
        python3 bench.py --workload vocoder --batch $b --steps 100 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/${tag}_b${b}_${v}_$i.json 2>/dev/null || exit 1
    rm -f gpurun_out/${tag}_b${b}_${v}_$i/run_kernel_trace.csv
  done
done
done
