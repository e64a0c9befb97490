# Stage1 head with input_conv composed into ConvT1 vs the two-layer head
# (M2_HEAD_INCONV=1): the vocoder GPU tests first, then kernel stats of the
# headline vocoder, arms alternated on one box.
# Table: python tools/probe/ab_table.py hc head
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_head_comp.py tests/test_gpu_tailp.py tests/test_gpu_tailp2.py tests/test_gpu_parity.py tests/test_gpu_sharding_streaming.py tests/test_gpu_range.py -x -q --timeout 200 --timeout-method thread > gpurun_out/hc_tests.log 2>&1 || { tail -n 40 gpurun_out/hc_tests.log; exit 1; }
tail -n 1 gpurun_out/hc_tests.log
for i in 1 2; do
for v in comp inconv; do
  unset M2_HEAD_INCONV
  if [ $v = inconv ]; then export M2_HEAD_INCONV=1; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hc_${v}_$i -o run -- \
      python3 bench.py --steps 100 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/hc_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/hc_${v}_$i/run_kernel_trace.csv
done
done
unset M2_HEAD_INCONV
for shape in 8x500 16x2600; do
for i in 1 2; do
for v in six seven; do
  unset M2_TAILP2_SEVEN
  if [ $v = seven ]; then export M2_TAILP2_SEVEN=1; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/o2_${shape}_${v}_$i -o run -- \
      python3 bench.py --workload s2_vocoder --s2-shape $shape --steps 50 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/o2_${shape}_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/o2_${shape}_${v}_$i/run_kernel_trace.csv
done
done
done
