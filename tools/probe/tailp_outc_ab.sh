# Stage1 tail, six-layer form (composed ResBlock4-conv2 + output_conv) vs the
# seven-layer form (M2_TAILP_SEVEN=1): the tail tests and the vocoder parity
# tests first, then kernel stats of the headline vocoder, arms alternated on
# one box.  Table: python tools/probe/ab_table.py outc tailp
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tailp.py tests/test_gpu_parity.py tests/test_gpu_sharding_streaming.py tests/test_gpu_range.py -x -q --timeout 200 --timeout-method thread > gpurun_out/outc_tests.log 2>&1 || { tail -n 40 gpurun_out/outc_tests.log; exit 1; }
tail -n 1 gpurun_out/outc_tests.log
for i in 1 2; do
for v in six seven; do
  unset M2_TAILP_SEVEN
  if [ $v = seven ]; then export M2_TAILP_SEVEN=1; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/outc_${v}_$i -o run -- \
      python3 bench.py --steps 100 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/outc_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/outc_${v}_$i/run_kernel_trace.csv
done
done
