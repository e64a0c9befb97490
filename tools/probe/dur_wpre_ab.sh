# Duration kernel: conv weights requested at kernel start (new) vs inside the
# conv loops (old library): parity tests, then kernel stats of the stage1
# pipeline and the stage2 B=8 per-GPU share (s2_b64 at --s2-batch 8 is the
# bench's s2_b8_per_gpu_share line), arms alternated on one box.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharding_streaming.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dw_tests.log 2>&1 || { tail -n 30 gpurun_out/dw_tests.log; exit 1; }
tail -n 1 gpurun_out/dw_tests.log
for i in 1 2; do
for v in new old; do
  unset M2TTS_HIP_LIB
  if [ $v = old ]; then export M2TTS_HIP_LIB=tools/probe/libm2_dur_old.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dw_${v}_$i -o run -- \
      python3 bench.py --workload pipeline --steps 100 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/dw_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/dw_${v}_$i/run_kernel_trace.csv
done
done
