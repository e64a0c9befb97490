# Round 6: pipeline tests (fixture test new), the two-lane kernel trace of the
# B=8 share (front / back overlap), the bench on plain streams.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharding_streaming.py tests/test_gpu_device_T.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06o_tests.log 2>&1 || { tail -n 30 gpurun_out/r06o_tests.log; exit 1; }
tail -n 1 gpurun_out/r06o_tests.log
d=gpurun_out/r06o_pipe_trace
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/pipe_trace.py 2 > $d.log 2>&1 || { tail -n 20 $d.log; exit 1; }
python3 tools/probe/pipe_trace.py --summarize $d/run_kernel_trace.csv > gpurun_out/r06o_pipe_trace.txt || exit 1
rm -f $d/run_kernel_trace.csv
head -30 gpurun_out/r06o_pipe_trace.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06o_bench_driver.json 2> gpurun_out/r06o_bench_driver.err || exit 1
grep "ms/step" gpurun_out/r06o_bench_driver.err
