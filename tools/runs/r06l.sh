# Round 6: ShardedPipeline back-stream priority A/B (B=8 and B=64), pipeline tests.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/probe/pipe_prio_ab.py > gpurun_out/r06l_prio_ab.txt 2>&1 || { tail -n 30 gpurun_out/r06l_prio_ab.txt; exit 1; }
cat gpurun_out/r06l_prio_ab.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_T.py tests/test_gpu_sharding_streaming.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06l_tests.log 2>&1 || { tail -n 30 gpurun_out/r06l_tests.log; exit 1; }
tail -n 1 gpurun_out/r06l_tests.log
