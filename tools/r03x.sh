# Round 3 A/B: wave-priority stagger in the query-split attention (M2_TFL_PRIO=1) - parity and decoder layer times.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
M2_TFL_PRIO=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_device_T.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03x_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03x_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  for B in 64 16; do
    S=100; [ $B = 16 ] && S=520
    M2_TFL_PRIO=$v timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/x_$B -o run -- python3 tools/probe/s2_small_trace.py $B one $S > gpurun_out/x_$B.log 2>&1 || exit 1
    python3 tools/probe/s2_small_trace.py --summarize gpurun_out/x_$B/run_kernel_trace.csv 10 > gpurun_out/x_${B}_$v.txt || exit 1
    rm -f gpurun_out/x_$B/run_kernel_trace.csv
    echo "prio $v B $B: $(head -1 gpurun_out/x_${B}_$v.txt) | $(grep 'layer_kernel<96, false' gpurun_out/x_${B}_$v.txt | awk '{print $2}' | tr '\n' ' ')" | tee -a gpurun_out/r03x_ab.txt
  done
done
