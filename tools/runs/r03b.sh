# Round 3: first run of the one-launch transformer layers: their tests, the
# parity suite, then the B=8 / B=64 kernel traces and the driver-form bench.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03b_tfl.log 2>&1
rc=$?; tail -3 gpurun_out/r03b_tfl.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03b_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/probe/s2_small_trace.sh &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03b_bench_driver.json 2> gpurun_out/r03b_bench_driver.err
