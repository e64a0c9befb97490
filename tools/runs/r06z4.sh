# Round 6, re-entry: the GPU suite and a driver-form bench with the two-phase
# exact-f32 tail defaults and the sparser roofline event sampling.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06z4_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/r06z4_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/r06z4_gpu_tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06z4_bench_driver.json 2> gpurun_out/r06z4_bench_driver.err || { tail -n 20 gpurun_out/r06z4_bench_driver.err; exit 1; }
grep "ms/step" gpurun_out/r06z4_bench_driver.err
