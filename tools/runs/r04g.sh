# Round 4: 128-row decoder tiles (layer_kernel RB = 8, attention_q128):
# tile tests of every form, in-process A/Bs against the default tiles at the
# long-form and the mid-size decoder grids, long-form kernel trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04g_tf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04g_tf_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_RB unset,8 s2 128 520 4 2 > gpurun_out/r04g_rb8_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r04g_rb8_ab_lf.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_RB unset,8 s2 16 520 6 4 > gpurun_out/r04g_rb8_ab_16.txt 2>&1 || exit 1
cat gpurun_out/r04g_rb8_ab_16.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_RB unset,8 s2 64 100 6 10 > gpurun_out/r04g_rb8_ab_64.txt 2>&1 || exit 1
cat gpurun_out/r04g_rb8_ab_64.txt
for v in 8 0; do
  M2_TFL_RB=$v timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04g_lf_rb$v -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > gpurun_out/r04g_lf_rb$v.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize gpurun_out/r04g_lf_rb$v/run_kernel_trace.csv 3 > gpurun_out/r04g_lf_rb$v.txt || exit 1
  rm -f gpurun_out/r04g_lf_rb$v/run_kernel_trace.csv
  echo "== rb=$v"; grep -E "span|layer_kernel" gpurun_out/r04g_lf_rb$v.txt
done
