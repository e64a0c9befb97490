# Tail role layouts A/B: parity on the vocoder tests, then kernel stats of the
# headline bench per variant library (built by make OBJDIR=build_<v> ...).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in s4 s5 s0; do
  L=m2-tts_amd/csrc/build_$v/libm2tts_hip_$v.so
  M2TTS_HIP_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
      -k "vocoder" > gpurun_out/split_${v}_tests.log 2>&1 || { tail -5 gpurun_out/split_${v}_tests.log; exit 1; }
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/split_$v -o run -- \
      python3 bench.py --steps 100 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/split_${v}_bench.json 2>/dev/null || exit 1
  rm -f gpurun_out/split_$v/run_kernel_trace.csv
done
