# Round 3 A/B: 64-row tiles for the first LN1 -> QKV launch (M2_TFL_FIRST_RB=4) - parity and kernel times.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
M2_TFL_FIRST_RB=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_device_T.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03w_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03w_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 2 4 2 4; do
  for B in 64 128; do
    S=100; [ $B = 128 ] && S=520
    M2_TFL_FIRST_RB=$v timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/w_$B -o run -- python3 tools/probe/s2_small_trace.py $B one $S > gpurun_out/w_$B.log 2>&1 || exit 1
    python3 tools/probe/s2_small_trace.py --summarize gpurun_out/w_$B/run_kernel_trace.csv 10 > gpurun_out/w_${B}_$v.txt || exit 1
    rm -f gpurun_out/w_$B/run_kernel_trace.csv
    echo "rb $v B $B: $(head -1 gpurun_out/w_${B}_$v.txt) first: $(grep 'first_kernel<96, 2' gpurun_out/w_${B}_$v.txt)" | tee -a gpurun_out/r03w_ab.txt
  done
done
