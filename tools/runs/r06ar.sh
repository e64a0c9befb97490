# Round 6: with form 12 in place, the decoder tile choice at the smaller
# grids - M2_TFL_RB_UNMASKED unset / 2 / 4 (64-row form-12 tiles) on stage1
# B=32 S=100 (configs[1]'s inference) and stage2 B=8 S=100 (configs[3]'s
# per-GPU share), B=16 S=100.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_RB_UNMASKED unset,2,4 s1 32 100 8 30 > gpurun_out/r06ar_ab_s1.txt 2>&1 || exit 1
cat gpurun_out/r06ar_ab_s1.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_RB_UNMASKED unset,2,4 s2 8 100 8 30 > gpurun_out/r06ar_ab_s2_8.txt 2>&1 || exit 1
cat gpurun_out/r06ar_ab_s2_8.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_RB_UNMASKED unset,2,4 s2 16 100 8 30 > gpurun_out/r06ar_ab_s2_16.txt 2>&1 || exit 1
cat gpurun_out/r06ar_ab_s2_16.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_RB_UNMASKED unset,2,4 s2 64 100 6 10 > gpurun_out/r06ar_ab_s2_64.txt 2>&1 || exit 1
cat gpurun_out/r06ar_ab_s2_64.txt
