# 4- vs 8-wave fused transformer layers: parity (default rule and forced 8),
# kernel trace of stage2 inference at B=8 / 64, bench A/B of the pipeline and
# the configs[3] per-GPU share.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tfw_tests.log 2>&1 || { tail -n 20 gpurun_out/tfw_tests.log; exit 1; }
M2_TF_WAVES=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tfw_tests8.log 2>&1 || { tail -n 20 gpurun_out/tfw_tests8.log; exit 1; }
tail -n 1 gpurun_out/tfw_tests.log gpurun_out/tfw_tests8.log
for B in 8 64; do
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tfw_b$B -o run -- python3 tools/probe/s2_small_trace.py $B > gpurun_out/tfw_b$B.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/tfw_b$B/run_kernel_trace.csv > gpurun_out/tfw_b$B.txt || exit 1
rm -f gpurun_out/tfw_b$B/run_kernel_trace.csv
done
for i in 1 2; do
  for w in 4 0; do
    M2_TF_WAVES=$w timeout -k 10 200 python bench.py --workload pipeline --no-extras --no-cpu-baseline --steps 300 --warmup 20 > gpurun_out/tfw_pipe_w${w}_$i.json 2>/dev/null || exit 1
    M2_TF_WAVES=$w timeout -k 10 200 python bench.py --workload s2_b64 --no-extras --no-cpu-baseline --steps 100 --warmup 20 > gpurun_out/tfw_s2b64_w${w}_$i.json 2>/dev/null || exit 1
  done
done
