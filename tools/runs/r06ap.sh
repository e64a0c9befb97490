# Round 6: form 12 - in-process A/B of priority to the lagging SIMD partner
# (M2_TFL_QPRIO=1: each wave posts its chunk index in LDS and sets s_setprio
# by its partner's).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
M2_TFL_QPRIO=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06ap_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06ap_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/probe/env_ab.py M2_TFL_QPRIO 0,1 s2 128 520 6 2 > gpurun_out/r06ap_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r06ap_ab_lf.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QPRIO 0,1 s2 16 520 6 4 > gpurun_out/r06ap_ab_16.txt 2>&1 || exit 1
cat gpurun_out/r06ap_ab_16.txt
