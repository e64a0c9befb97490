# Round 6: host cost breakdown of ShardedPipeline.submit (cProfile), then the stress-flip probe.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/probe/pipe_host.py --profile > gpurun_out/r06g_submit_prof.txt 2>&1 || { tail -n 30 gpurun_out/r06g_submit_prof.txt; exit 1; }
head -45 gpurun_out/r06g_submit_prof.txt
bash tools/runs/r06f.sh
