# Round 6: host cost of ShardedPipeline submit / wait at the B=8 share.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/probe/pipe_host.py 200 > gpurun_out/r06e_pipe_host.txt 2>&1 || { tail -n 30 gpurun_out/r06e_pipe_host.txt; exit 1; }
cat gpurun_out/r06e_pipe_host.txt
timeout -k 10 300 python3 -u tools/probe/cumask_share2.py > gpurun_out/r06e_cumask2.txt 2>&1 || { tail -n 30 gpurun_out/r06e_cumask2.txt; exit 1; }
head -3 gpurun_out/r06e_cumask2.txt
