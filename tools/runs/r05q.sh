# Round 5: the headline vocoder's kernel time line with no profiling events
# (tools/probe/voc_gaps.py), summarised as in r05o.sh.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05q -o run -- python3 tools/probe/voc_gaps.py 200 > gpurun_out/r05q.log 2>&1 || exit 1
sed -n '/^import csv/,/^PY$/p' tools/runs/r05o.sh | sed '$d' > /tmp/gaps.py
TAG=r05q python3 /tmp/gaps.py | tee gpurun_out/r05q_gaps.txt
rm -f gpurun_out/r05q/run_kernel_trace.csv
