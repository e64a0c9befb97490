# Embedding / frame expansion fused into the first layer's LN1 -> QKV: the -m gpu
# suite, the stage2 B=8 kernel trace, bench pipeline + s2_b64.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ff_tests.log 2>&1 || { tail -n 30 gpurun_out/ff_tests.log; exit 1; }
tail -n 1 gpurun_out/ff_tests.log
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ff_b8 -o run -- python3 tools/probe/s2_small_trace.py 8 > gpurun_out/ff_b8.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/ff_b8/run_kernel_trace.csv > gpurun_out/ff_b8.txt || exit 1
rm -f gpurun_out/ff_b8/run_kernel_trace.csv
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload pipeline --no-extras --no-cpu-baseline --steps 300 --warmup 20 > gpurun_out/ff_pipe_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --workload s2_b64 --no-extras --no-cpu-baseline --steps 100 --warmup 20 > gpurun_out/ff_s2b64_$i.json 2>/dev/null || exit 1
done
