set -u
mkdir -p gpurun_out
bash tools/probe/att_round.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharding_streaming.py -m gpu -x -q -k s2 --timeout 120 --timeout-method thread > gpurun_out/s2_after_cache.log 2>&1
