# Round 3: query-split attention with two query blocks per wave (attention_qsplit2) - parity, in-process A/B, long-form trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03ab_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_T.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ab_tests2.log 2>&1
rc=$?; tail -3 gpurun_out/r03ab_tests2.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r03ab_ab.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 0,1 s2 64 100 6 20 >> gpurun_out/r03ab_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 0,1 s2 16 520 5 4 >> gpurun_out/r03ab_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 0,1 s2 128 520 3 2 >> gpurun_out/r03ab_ab.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r03ab_ab.txt | cut -c1-110
for v in 0 1; do
M2_TFL_QS2=$v timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_$v -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > gpurun_out/ab_$v.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/ab_$v/run_kernel_trace.csv 3 > gpurun_out/r03ab_b128_qs$v.txt || exit 1
rm -f gpurun_out/ab_$v/run_kernel_trace.csv
grep -E "span|layer_kernel" gpurun_out/r03ab_b128_qs$v.txt
done
