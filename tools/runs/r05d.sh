# Round 5: scaled-weight stress parity (tests/test_gpu_stress.py) and the
# stage1 pipeline's kernel trace (configs[2], B=32 S=100).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stress.py -q --timeout 200 --timeout-method thread > gpurun_out/r05d_stress.log 2>&1
rc=$?; tail -15 gpurun_out/r05d_stress.log
d=gpurun_out/r05d_tr_s1_32
M2_TRACE_STAGE=s1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 32 one 100 > $d.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 20 > $d.txt || exit 1
rm -f $d/run_kernel_trace.csv
cat $d.txt
exit $rc
