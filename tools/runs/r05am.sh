# Round 5: the 32-row first (LN1 -> QKV) launch at H <= 64 with all of a
# wave's QKV strips requested at the start, against the previous commit's
# build (build_base): layer tests, B=8 S=100 stage2 traces, stage1 pipeline
# kernel stats, alternated twice.
set -u
tag=r05am
export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=m2-tts_amd/src/m2amd/libm2tts_hip.so
OLD=m2-tts_amd/csrc/build_base/libm2tts_hip_base.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_parity.py tests/test_gpu_device_T.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
for i in 1 2; do
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  d=gpurun_out/${tag}_tr8_${v}_$i
  M2TTS_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 8 dev 100 > $d.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 20 > $d.txt || exit 1
  rm -f $d/run_kernel_trace.csv
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_pipe_${v}_$i -o run -- \
      python3 bench.py --workload pipeline --steps 100 --warmup 20 --no-cpu-baseline --no-extras > gpurun_out/${tag}_pipe_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/${tag}_pipe_${v}_$i/run_kernel_trace.csv
done
done
