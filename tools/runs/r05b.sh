# (run at commit f29dcf2, where the split head existed behind M2_S2_HEAD_SPLIT)
# Round 5: the split stage2 head (M2_S2_HEAD_SPLIT) - parity, in-process A/B
# on the configs[3] share (B=8 S=100), B=64, long form, and a B=8 kernel trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_s2_head_split.py tests/test_gpu_range.py tests/test_gpu_head_comp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_S2_HEAD_SPLIT 0,1 s2 8 100 8 40 > gpurun_out/r05b_ab_8.txt 2>&1 || exit 1
cat gpurun_out/r05b_ab_8.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_S2_HEAD_SPLIT 0,1 s2 64 100 6 10 > gpurun_out/r05b_ab_64.txt 2>&1 || exit 1
cat gpurun_out/r05b_ab_64.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_S2_HEAD_SPLIT 0,1 s2 128 520 3 2 > gpurun_out/r05b_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r05b_ab_lf.txt
for v in 0 1; do
  d=gpurun_out/r05b_tr_8_split$v
  M2_S2_HEAD_SPLIT=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 8 dev 100 > $d.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 3 > $d.txt || exit 1
  rm -f $d/run_kernel_trace.csv
  head -16 $d.txt
done
