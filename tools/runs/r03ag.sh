# Round 3: 64-row first (LN1 -> QKV) launch for grids of >= 16 rounds (M2_TFL_FIRST_RB) - parity, A/B at long-form and B=64.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ag_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03ag_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r03ag_ab.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_FIRST_RB 2,4 s2 128 520 4 2 >> gpurun_out/r03ag_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_FIRST_RB 2,4 s2 16 520 5 4 >> gpurun_out/r03ag_ab.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r03ag_ab.txt | cut -c1-110
for v in 2 4; do
M2_TFL_FIRST_RB=$v timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ag_$v -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > gpurun_out/ag_$v.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/ag_$v/run_kernel_trace.csv 3 > gpurun_out/r03ag_b128_first$v.txt || exit 1
rm -f gpurun_out/ag_$v/run_kernel_trace.csv
cat gpurun_out/r03ag_b128_first$v.txt
done
