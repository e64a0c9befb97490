# Round-3 baseline on a fresh box: bench as the driver runs it, and the
# kernel trace of configs[3]'s per-GPU share (B=8) and of B=64.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03a_bench_driver.json 2> gpurun_out/r03a_bench_driver.err &&
bash tools/probe/s2_small_trace.sh
