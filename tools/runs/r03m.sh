# Round 3 re-entry: full GPU suite + smoke + default bench + vocoder/pipeline kernel stats on HEAD.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03m_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r03m_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03m_smoke.log 2>&1 || exit 1
cat gpurun_out/r03m_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03m_bench.json 2> gpurun_out/r03m_bench.err || exit 1
tail -c 3000 gpurun_out/r03m_bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03m_voc -o run -- python3 bench.py --no-cpu-baseline --no-extras --steps 50 --warmup 10 > gpurun_out/r03m_voc.log 2>&1 || exit 1
find gpurun_out/r03m_voc -name "*kernel_stats.csv" | head -3
