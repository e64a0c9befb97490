# Round 4: the wave-specialised attention with LDS-DMA staging (M2_TFL_QS2=9)
# against the current defaults (6 at head_dim 48, 4 at head_dim 32): every
# tile test, in-process A/Bs on stage2 (long-form, B=16 T=2600, B=64 T=500)
# and stage1 (B=32 S=100 = the pipeline line, B=128 S=100).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04n_tf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04n_tf_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 6,9 s2 128 520 4 2 > gpurun_out/r04n_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r04n_ab_lf.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 6,9 s2 16 520 6 4 > gpurun_out/r04n_ab_16.txt 2>&1 || exit 1
cat gpurun_out/r04n_ab_16.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 6,9 s2 64 100 6 10 > gpurun_out/r04n_ab_64.txt 2>&1 || exit 1
cat gpurun_out/r04n_ab_64.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 4,9 s1 32 100 8 30 > gpurun_out/r04n_ab_s1_32.txt 2>&1 || exit 1
cat gpurun_out/r04n_ab_s1_32.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 4,9 s1 128 100 6 10 > gpurun_out/r04n_ab_s1_128.txt 2>&1 || exit 1
cat gpurun_out/r04n_ab_s1_128.txt
