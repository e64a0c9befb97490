# Round 6: kernel trace of configs[4]'s workload on the final tree (stage2
# B=128 S=520 -> T=2600, one-call inference, unchunked vocoder): per-layer
# decoder launch times.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
d=gpurun_out/r06w_tr_128_one_520
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $d.log 2>&1 || { tail -n 20 $d.log; exit 1; }
python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 3 > gpurun_out/r06w_tr_128_one_520.txt || exit 1
rm -f $d/run_kernel_trace.csv
cat gpurun_out/r06w_tr_128_one_520.txt
