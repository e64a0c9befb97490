# Round 4: the first (LN1 -> QKV) launch's tile rows at configs[4] again
# (M2_TFL_FIRST_RB 4 default vs 2 / 1), in-process.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/probe/env_ab.py M2_TFL_FIRST_RB 4,2,1 s2 128 520 4 2 > gpurun_out/r04aa_first_rb.txt 2>&1 || exit 1
cat gpurun_out/r04aa_first_rb.txt
