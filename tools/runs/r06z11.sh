# Kernel traces on the final tree: the stage1 pipeline (configs[2], B=32
# S=100) and configs[3]'s B=8 share (stage2, one step at a time).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
d=gpurun_out/r06z11_tr_s1_32
M2_TRACE_STAGE=s1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 32 one 100 > $d.log 2>&1 || { tail -n 20 $d.log; exit 1; }
python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 20 > $d.txt || exit 1
rm -f $d/run_kernel_trace.csv
cat $d.txt
d=gpurun_out/r06z11_tr_s2_8
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 8 one 100 > $d.log 2>&1 || { tail -n 20 $d.log; exit 1; }
python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 20 > $d.txt || exit 1
rm -f $d/run_kernel_trace.csv
cat $d.txt
