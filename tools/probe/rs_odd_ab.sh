# Odd row strides (RS/16 odd) for the transposed convs' output buffers of the
# stage2 x3 head (u, h) and mid (u, h) vs the (RS/16) % 4 == 2 strides (old
# library): parity tests, then stage2 vocoder kernel stats, alternated.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_head_comp.py tests/test_gpu_tailp2.py tests/test_gpu_parity.py tests/test_gpu_sharding_streaming.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rs_tests.log 2>&1 || { tail -n 30 gpurun_out/rs_tests.log; exit 1; }
tail -n 1 gpurun_out/rs_tests.log
for shape in 8x500 16x2600; do
for i in 1 2; do
for v in new old; do
  unset M2TTS_HIP_LIB
  if [ $v = old ]; then export M2TTS_HIP_LIB=tools/probe/libm2_rs_old.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rs_${shape}_${v}_$i -o run -- \
      python3 bench.py --workload s2_vocoder --s2-shape $shape --steps 50 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/rs_${shape}_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/rs_${shape}_${v}_$i/run_kernel_trace.csv
done
done
done
