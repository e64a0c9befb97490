# Round 6: kernel trace of the stage1 pipeline (configs[2], B=32 S=100, one-call inference).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
d=gpurun_out/r06r_s1_pipe
M2_TRACE_STAGE=s1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 32 one 100 > $d.log 2>&1 || { tail -n 20 $d.log; exit 1; }
python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 20 > gpurun_out/r06r_s1_pipe.txt || exit 1
rm -f $d/run_kernel_trace.csv
cat gpurun_out/r06r_s1_pipe.txt
