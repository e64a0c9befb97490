# Round 6: CU-partitioned lanes feasibility (tools/probe/cumask_share.py).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/probe/cumask_share.py 32 48 64 96 > gpurun_out/r06b_cumask.txt 2>&1 || { tail -n 30 gpurun_out/r06b_cumask.txt; exit 1; }
cat gpurun_out/r06b_cumask.txt
