# Round 6: ShardedPipeline vs hardware-queue layout: GPU-side caller wait vs host wait.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/probe/pipe_queues.py torch hostwait > gpurun_out/r06p_q4.txt 2>&1 || { tail -n 30 gpurun_out/r06p_q4.txt; exit 1; }
cat gpurun_out/r06p_q4.txt


