#!/bin/bash
# GPU box: the -m gpu suite, then bench.py as the driver runs it and with its
# defaults.  Usage: tools/gpu_check.sh <tag>   (outputs under gpurun_out/)
set -u
tag=$1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench_driver.json 2> gpurun_out/${tag}_bench_driver.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench_default.json 2> gpurun_out/${tag}_bench_default.err
