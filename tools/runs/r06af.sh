# Round 6: attention form 13 (form 12 with each wave's next chunk moved into
# a private LDS slot by LDS-DMA a whole iteration ahead) - tests, in-process
# A/Bs against 9 and 12, and a configs[4] kernel trace on 13.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_range.py -k "4q13 or scores_large" -x -q --timeout 120 --timeout-method thread > gpurun_out/r06af_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06af_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 9,12,13 s2 128 520 4 2 > gpurun_out/r06af_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r06af_ab_lf.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 9,12,13 s2 16 520 6 4 > gpurun_out/r06af_ab_16.txt 2>&1 || exit 1
cat gpurun_out/r06af_ab_16.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 9,12,13 s2 64 100 6 10 > gpurun_out/r06af_ab_64.txt 2>&1 || exit 1
cat gpurun_out/r06af_ab_64.txt
d=gpurun_out/r06af_tr_q13
export M2_TFL_QS2=13
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $d.log 2>&1 || { tail -n 20 $d.log; exit 1; }
python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 3 > gpurun_out/r06af_tr_q13.txt || exit 1
rm -f $d/run_kernel_trace.csv
cat gpurun_out/r06af_tr_q13.txt
