# Round 6: form 12 with the out projection's strip and residual rows requested
# before the merge; in-process A/B of a barrier every n chunks (M2_TFL_QBAR)
# against none, configs[4] trace, stamps build.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_range.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06an_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06an_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/probe/env_ab.py M2_TFL_QBAR 0,1,2,4,8 s2 128 520 4 2 > gpurun_out/r06an_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r06an_ab_lf.txt
d=gpurun_out/r06an_tr_lf
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $d.log 2>&1 || { tail -n 20 $d.log; exit 1; }
python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 3 > gpurun_out/r06an_tr_lf.txt || exit 1
rm -f $d/run_kernel_trace.csv
cat gpurun_out/r06an_tr_lf.txt
