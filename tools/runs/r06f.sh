# Round 6: which path writes the far samples of the x4 stress test (item 6).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/probe/stress_flips.py 4 > gpurun_out/r06f_flips.txt 2>&1 || { tail -n 30 gpurun_out/r06f_flips.txt; exit 1; }
cat gpurun_out/r06f_flips.txt
timeout -k 10 300 python3 -u tools/probe/stress_flips.py 2 > gpurun_out/r06f_flips2.txt 2>&1 || { tail -n 30 gpurun_out/r06f_flips2.txt; exit 1; }
cat gpurun_out/r06f_flips2.txt
