# Round 6: attention_tile (16 / 32-row tiles) with the two waves of each SIMD
# taking the issue priority in turn (M2_TFL_TPRIO=1) - in-process A/Bs at
# configs[3]'s share (stage2 B=8 S=100), stage1 B=32 S=100, stage2 B=16 S=100.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
M2_TFL_TPRIO=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06au_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06au_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_TPRIO 0,1 s2 8 100 8 30 > gpurun_out/r06au_ab_s2_8.txt 2>&1 || exit 1
cat gpurun_out/r06au_ab_s2_8.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_TPRIO 0,1 s1 32 100 8 30 > gpurun_out/r06au_ab_s1.txt 2>&1 || exit 1
cat gpurun_out/r06au_ab_s1.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_TPRIO 0,1 s2 16 100 8 30 > gpurun_out/r06au_ab_s2_16.txt 2>&1 || exit 1
cat gpurun_out/r06au_ab_s2_16.txt
