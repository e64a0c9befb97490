# Round 6: ShardedPipeline vs hardware-queue assignment (tools/probe/pipe_queues.py).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/probe/pipe_queues.py torch lo/hi hi/lo > gpurun_out/r06m_queues.txt 2>&1 || { tail -n 30 gpurun_out/r06m_queues.txt; exit 1; }
cat gpurun_out/r06m_queues.txt
