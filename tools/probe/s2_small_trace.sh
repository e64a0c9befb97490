# Kernel traces of stage2 inference at B=8 / B=64 (S=100): MODE = two (host-T
# front + back), one (m2_inference), dev (sharded flow, device-T).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
MODE=${1:-two}
for B in 8 64; do
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2t_b$B -o run -- python3 tools/probe/s2_small_trace.py $B $MODE > gpurun_out/s2t_b$B.log 2>&1 || exit 1
python3 tools/probe/s2_small_trace.py --summarize gpurun_out/s2t_b$B/run_kernel_trace.csv > gpurun_out/s2t_${MODE}_b$B.txt || exit 1
rm -f gpurun_out/s2t_b$B/run_kernel_trace.csv
done
