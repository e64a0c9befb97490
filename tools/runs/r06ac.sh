# Round 6: front-half tilings for the pipelined B=8 share (tools/probe/front_tiles.py).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/probe/front_tiles.py --dec > gpurun_out/r06ac_front_tiles.txt 2>&1 || { tail -n 30 gpurun_out/r06ac_front_tiles.txt; exit 1; }
cat gpurun_out/r06ac_front_tiles.txt
