# Round 6: ShardedPipeline vs hardware-queue count: the queue-rotation probe
# with the box default (4) and with GPU_MAX_HW_QUEUES=8.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/probe/pipe_queues.py torch > gpurun_out/r06n_q4.txt 2>&1 || { tail -n 30 gpurun_out/r06n_q4.txt; exit 1; }
cat gpurun_out/r06n_q4.txt
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 -u tools/probe/pipe_queues.py torch > gpurun_out/r06n_q8.txt 2>&1 || { tail -n 30 gpurun_out/r06n_q8.txt; exit 1; }
cat gpurun_out/r06n_q8.txt
