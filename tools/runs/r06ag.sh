# Round 6: form 12 variants - 14 both pairs' QK^T first, 15 s_setprio around
# the MFMA groups, 16 both - in-process A/Bs against 12.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 12,14,15,16 s2 128 520 4 2 > gpurun_out/r06ag_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r06ag_ab_lf.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 12,14,15,16 s2 16 520 6 4 > gpurun_out/r06ag_ab_16.txt 2>&1 || exit 1
cat gpurun_out/r06ag_ab_16.txt
