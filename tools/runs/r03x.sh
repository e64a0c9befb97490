# Round 3 in-process A/Bs: wave-priority stagger (M2_TFL_PRIO) and 64-row first-launch tiles (M2_TFL_FIRST_RB).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
M2_TFL_PRIO=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_device_T.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03x_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03x_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r03x_ab.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_PRIO 0,1 s2 64 100 8 30 >> gpurun_out/r03x_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_PRIO 0,1 s2 16 520 6 5 >> gpurun_out/r03x_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_PRIO 0,1 s1 32 100 8 40 >> gpurun_out/r03x_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_FIRST_RB 2,4 s2 64 100 8 30 >> gpurun_out/r03x_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_FIRST_RB 2,4 s2 16 520 6 5 >> gpurun_out/r03x_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_FIRST_RB 2,4 s1 32 100 8 40 >> gpurun_out/r03x_ab.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r03x_ab.txt | cut -c1-120
