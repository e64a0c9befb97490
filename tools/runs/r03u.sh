set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/probe/shard_gloo_probe.py 64 100 all 1 2>&1 | tee gpurun_out/r03u_all.txt
timeout -k 10 120 python -u tools/probe/shard_gloo_probe.py 64 100 0 1 2>&1 | tee gpurun_out/r03u_g0.txt
