# Round 6: DMA loaders with per-strip descriptors - tail / streaming (incl.
# U2 past 2 GB) / parity / range tests.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tailp.py tests/test_gpu_tailp2.py tests/test_gpu_sharding_streaming.py tests/test_gpu_parity.py tests/test_gpu_range.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06x_tests.log 2>&1 || { tail -n 30 gpurun_out/r06x_tests.log; exit 1; }
tail -n 1 gpurun_out/r06x_tests.log
grep -i "past_2gb" gpurun_out/r06x_tests.log || true
