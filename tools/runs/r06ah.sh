# Round 6: the key-quarter form (12) as the head_dim-48 default, form 9
# removed - full GPU suite, stage1 A/B of 12 against its default (4) on
# 64-row grids, and the default bench (every line).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06ah_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/r06ah_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/r06ah_gpu_tests.log
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 4,12 s1 128 130 6 6 > gpurun_out/r06ah_ab_s1_128.txt 2>&1 || exit 1
cat gpurun_out/r06ah_ab_s1_128.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 4,12 s1 32 520 6 6 > gpurun_out/r06ah_ab_s1_32l.txt 2>&1 || exit 1
cat gpurun_out/r06ah_ab_s1_32l.txt
timeout -k 10 500 python -u bench.py > gpurun_out/r06ah_bench.json 2> gpurun_out/r06ah_bench.err || exit 1
grep "ms/step" gpurun_out/r06ah_bench.err
