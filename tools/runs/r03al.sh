# Round 3: lean softmax in the one-block query-split attention (M2_TFL_QS2=4) - parity, in-process A/B (stage1 B=32 pipeline).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03al_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03al_tests.log; [ $rc -eq 0 ] || exit $rc
M2_TFL_QS2=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03al_tests2.log 2>&1
rc=$?; tail -2 gpurun_out/r03al_tests2.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r03al_ab.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 0,4 s1 32 100 10 40 >> gpurun_out/r03al_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 3,4 s2 16 520 6 4 >> gpurun_out/r03al_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 3,4 s2 64 100 6 20 >> gpurun_out/r03al_ab.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r03al_ab.txt | cut -c1-110
