# Round 6 final record on the composed exact-f32 head + two-phase tail tree:
# the GPU suite, smoke, a driver-form bench, the exact-f32 kernel stats.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06z8_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/r06z8_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/r06z8_gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06z8_smoke.log 2>&1 || { tail -n 20 gpurun_out/r06z8_smoke.log; exit 1; }
tail -n 1 gpurun_out/r06z8_smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06z8_bench_driver.json 2> gpurun_out/r06z8_bench_driver.err || { tail -n 20 gpurun_out/r06z8_bench_driver.err; exit 1; }
grep "ms/step" gpurun_out/r06z8_bench_driver.err
d=gpurun_out/prof_r06z8_f32
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/probe/voc_gaps.py 400 f32 > $d.log 2>&1 || { tail -n 20 $d.log; exit 1; }
rm -f $d/run_kernel_trace.csv
cp $d/run_kernel_stats.csv gpurun_out/r06z8_f32_kernel_stats.csv
cut -d, -f1-4 gpurun_out/r06z8_f32_kernel_stats.csv | cut -c1-60,200-
