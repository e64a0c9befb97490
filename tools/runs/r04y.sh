# Round 4: the ping-pong form (6) with the base in the tail k-step, against
# the wave-specialised default (9): tile tests, in-process A/Bs.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread -k "4q6 or auto" > gpurun_out/r04y_tf_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04y_tf_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 9,6 s2 128 520 4 2 > gpurun_out/r04y_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r04y_ab_lf.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 9,6 s2 16 520 6 4 > gpurun_out/r04y_ab_16.txt 2>&1 || exit 1
cat gpurun_out/r04y_ab_16.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 9,6 s2 64 100 6 10 > gpurun_out/r04y_ab_64.txt 2>&1 || exit 1
cat gpurun_out/r04y_ab_64.txt
