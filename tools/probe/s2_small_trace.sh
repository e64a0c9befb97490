set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for B in 8 64; do
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2t_b$B -o run -- python3 tools/probe/s2_small_trace.py $B > gpurun_out/s2t_b$B.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/s2t_b$B/run_kernel_trace.csv > gpurun_out/s2t_b$B.txt || exit 1
rm -f gpurun_out/s2t_b$B/run_kernel_trace.csv
done
