# Round 3: 30-phoneme duration tiles for large grids (M2_DUR_RB) - parity, in-process A/B, long-form trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_T.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03af_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03af_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r03af_ab.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_DUR_RB 1,2 s2 64 100 6 20 >> gpurun_out/r03af_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_DUR_RB 1,2 s1 32 100 8 40 >> gpurun_out/r03af_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_DUR_RB 1,2 s2 128 520 3 2 >> gpurun_out/r03af_ab.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r03af_ab.txt | cut -c1-110
for v in 1 2; do
M2_DUR_RB=$v timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/af_$v -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > gpurun_out/af_$v.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/af_$v/run_kernel_trace.csv 3 > gpurun_out/r03af_b128_rb$v.txt || exit 1
rm -f gpurun_out/af_$v/run_kernel_trace.csv
grep -E "span|duration" gpurun_out/r03af_b128_rb$v.txt
M2_DUR_RB=$v timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/af64_$v -o run -- python3 tools/probe/s2_small_trace.py 64 one > gpurun_out/af64_$v.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/af64_$v/run_kernel_trace.csv > gpurun_out/r03af_b64_rb$v.txt || exit 1
rm -f gpurun_out/af64_$v/run_kernel_trace.csv
grep -E "span|duration" gpurun_out/r03af_b64_rb$v.txt
done
