# Round 6: split-stream pipeline of the B=8 share with stream priorities (raw calls).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/probe/cumask_share2.py --prio > gpurun_out/r06j_prio.txt 2>&1 || { tail -n 30 gpurun_out/r06j_prio.txt; exit 1; }
cat gpurun_out/r06j_prio.txt
