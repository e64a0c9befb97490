# Round 3: ShardedPipeline depth sweep (global batches in flight) for the B=8 per-GPU share and B=64 at world 1.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r03z_depth.txt
timeout -k 10 300 python -u tools/probe/depth_sweep.py 8 100 1,2,3,4 6 40 >> gpurun_out/r03z_depth.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/depth_sweep.py 64 100 1,2,3 5 20 >> gpurun_out/r03z_depth.txt 2>&1 || exit 1
grep depth gpurun_out/r03z_depth.txt
