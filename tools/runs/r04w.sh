# Round 4: persistent duration tiles on large grids (M2_DUR_PERS): tests
# (bit-identical front buffers, oracle), in-process A/Bs.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_T.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04w_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04w_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_DUR_PERS 0,1 s2 128 520 4 2 > gpurun_out/r04w_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r04w_ab_lf.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_DUR_PERS 0,1 s1 128 100 6 10 > gpurun_out/r04w_ab_s1_128.txt 2>&1 || exit 1
cat gpurun_out/r04w_ab_s1_128.txt
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04w_tr -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > gpurun_out/r04w_tr.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/r04w_tr/run_kernel_trace.csv 3 > gpurun_out/r04w_tr.txt || exit 1
rm -f gpurun_out/r04w_tr/run_kernel_trace.csv
head -10 gpurun_out/r04w_tr.txt
