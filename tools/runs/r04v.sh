# Round 4: the default range policy's per-call cost by guard-launch grid,
# timed like the headline (tools/probe/redo_cost.py).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/probe/redo_cost.py > gpurun_out/r04v_redo_cost.txt 2>&1 || exit 1
cat gpurun_out/r04v_redo_cost.txt
