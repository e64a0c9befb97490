# Round 6: host_wait default - pipeline tests and the driver-form bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharding_streaming.py tests/test_gpu_device_T.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06q_tests.log 2>&1 || { tail -n 30 gpurun_out/r06q_tests.log; exit 1; }
tail -n 1 gpurun_out/r06q_tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06q_bench_driver.json 2> gpurun_out/r06q_bench_driver.err || exit 1
grep "ms/step" gpurun_out/r06q_bench_driver.err
timeout -k 10 300 python3 -u tools/probe/pipe_host.py 200 > gpurun_out/r06q_pipe_host.txt 2>&1 || { tail -n 30 gpurun_out/r06q_pipe_host.txt; exit 1; }
cat gpurun_out/r06q_pipe_host.txt
