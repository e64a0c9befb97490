# Round 3: lean-softmax two-block query-split attention (M2_TFL_QS2=3: C = -m, row sums by MFMA) - parity, in-process A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03aj_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03aj_tests.log; [ $rc -eq 0 ] || exit $rc
M2_TFL_QS2=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharding_streaming.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03aj_tests2.log 2>&1
rc=$?; tail -2 gpurun_out/r03aj_tests2.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r03aj_ab.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 2,3 s2 128 520 4 2 >> gpurun_out/r03aj_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 2,3 s2 16 520 6 4 >> gpurun_out/r03aj_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 2,3 s2 64 100 6 20 >> gpurun_out/r03aj_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 0,3 s1 32 100 8 40 >> gpurun_out/r03aj_ab.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r03aj_ab.txt | cut -c1-110
M2_TFL_QS2=3 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/aj -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > gpurun_out/aj.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/aj/run_kernel_trace.csv 3 > gpurun_out/r03aj_b128_qs3.txt || exit 1
rm -f gpurun_out/aj/run_kernel_trace.csv
cat gpurun_out/r03aj_b128_qs3.txt
