# Round 4: the software-pipelined lean query-split attention (M2_TFL_QS2=5):
# tile tests of every form, in-process A/B against the lean two-block form on
# the long-form step, and a kernel trace of the long-form decoder layers.
set -u
TAG=${1:-d}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread -k "4q5 or 4q3" > gpurun_out/r04${TAG}_tf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04${TAG}_tf_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/probe/env_ab.py M2_TFL_QS2 3,5 s2 128 520 4 2 > gpurun_out/r04${TAG}_qs2_ab.txt 2>&1 || exit 1
cat gpurun_out/r04${TAG}_qs2_ab.txt
for i in 1 2; do for v in 3 5; do
  M2_TFL_QS2=$v timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04${TAG}_lf_q$v$i -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > gpurun_out/r04${TAG}_lf_q$v$i.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize gpurun_out/r04${TAG}_lf_q$v$i/run_kernel_trace.csv 3 > gpurun_out/r04${TAG}_lf_q$v$i.txt || exit 1
  rm -f gpurun_out/r04${TAG}_lf_q$v$i/run_kernel_trace.csv
  echo "== qs2=$v $i"; grep -E "span|layer_kernel" gpurun_out/r04${TAG}_lf_q$v$i.txt
done; done
