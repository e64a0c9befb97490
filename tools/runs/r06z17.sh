# Round 6 closing record on the final tree: GPU suite, smoke, driver-form and
# default benches, the headline kernel stats.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06z17_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/r06z17_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/r06z17_gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06z17_smoke.log 2>&1 || { tail -n 20 gpurun_out/r06z17_smoke.log; exit 1; }
tail -n 1 gpurun_out/r06z17_smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06z17_bench_driver.json 2> gpurun_out/r06z17_bench_driver.err || { tail -n 20 gpurun_out/r06z17_bench_driver.err; exit 1; }
grep "ms/step" gpurun_out/r06z17_bench_driver.err
timeout -k 10 500 python -u bench.py > gpurun_out/r06z17_bench.json 2> gpurun_out/r06z17_bench.err || { tail -n 20 gpurun_out/r06z17_bench.err; exit 1; }
grep "ms/step" gpurun_out/r06z17_bench.err
d=gpurun_out/prof_r06z17
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 100 --warmup 100 --no-cpu-baseline --no-extras > $d.log 2>&1 || { tail -n 20 $d.log; exit 1; }
rm -f $d/run_kernel_trace.csv
cp $d/run_kernel_stats.csv gpurun_out/r06z17_headline_kernel_stats.csv
