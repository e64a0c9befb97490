# Round 6: pipeline / sharding tests after the input-conversion fix.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharding_streaming.py tests/test_gpu_device_T.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06z_tests.log 2>&1 || { tail -n 30 gpurun_out/r06z_tests.log; exit 1; }
tail -n 1 gpurun_out/r06z_tests.log
