# Round 5: attention form 11 (lean two-block + LDS-DMA staging + base in the
# tail k-step) - tile / range / stress tests, in-process A/B against 9.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_range.py tests/test_gpu_stress.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05e_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 9,11 s2 128 520 4 2 > gpurun_out/r05e_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r05e_ab_lf.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 9,11 s2 16 520 6 4 > gpurun_out/r05e_ab_16.txt 2>&1 || exit 1
cat gpurun_out/r05e_ab_16.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 9,11 s2 64 100 6 10 > gpurun_out/r05e_ab_64.txt 2>&1 || exit 1
cat gpurun_out/r05e_ab_64.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 4,11 s1 32 100 8 30 > gpurun_out/r05e_ab_s1.txt 2>&1 || exit 1
cat gpurun_out/r05e_ab_s1.txt
