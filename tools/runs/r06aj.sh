# Round 6: form 12 (two-MFMA tail) against temporary form 18 - the same with
# the row sums as per-lane fp32 adds of the exponentials instead of MFMAs on
# an all-ones fragment; tests with 18 forced, in-process A/Bs.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
M2_TFL_QS2=18 timeout -k 10 400 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_range.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06aj_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06aj_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 12,18 s2 128 520 4 2 > gpurun_out/r06aj_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r06aj_ab_lf.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 12,18 s2 16 520 6 4 > gpurun_out/r06aj_ab_16.txt 2>&1 || exit 1
cat gpurun_out/r06aj_ab_16.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 12,18 s2 64 100 6 10 > gpurun_out/r06aj_ab_64.txt 2>&1 || exit 1
cat gpurun_out/r06aj_ab_64.txt
