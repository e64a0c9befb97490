# Round 3: frame count fused into the duration kernel (sc1 hand-off to the last workgroup) - parity, in-process A/B, traces.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_T.py tests/test_gpu_parity.py tests/test_gpu_sharding_streaming.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03aa_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03aa_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r03aa_ab.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_DUR_COUNT 0,1 s2 8 100 8 40 >> gpurun_out/r03aa_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_DUR_COUNT 0,1 s1 32 100 8 40 >> gpurun_out/r03aa_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_DUR_COUNT 0,1 s2 64 100 6 20 >> gpurun_out/r03aa_ab.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r03aa_ab.txt | cut -c1-110
bash tools/probe/s2_small_trace.sh dev && cat gpurun_out/s2t_dev_b8.txt
