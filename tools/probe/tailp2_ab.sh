# Stage2 pipelined tail: its tests, the stage2 parity/sharding tests, then
# kernel stats of the stage2 vocoder workloads with the pipelined tail and
# with the x3 tail (M2_VOC_TAIL_X3=1), alternated.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tailp2.py tests/test_gpu_parity.py tests/test_gpu_sharding_streaming.py tests/test_gpu_range.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tp2_tests.log 2>&1 || { tail -n 30 gpurun_out/tp2_tests.log; exit 1; }
tail -n 1 gpurun_out/tp2_tests.log
for shape in 8x500 16x2600; do
for i in 1 2; do
for v in tp2 x3; do
  if [ $v = x3 ]; then export M2_VOC_TAIL_X3=1; else unset M2_VOC_TAIL_X3; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tp2_${v}_${shape}_$i -o run -- \
      python3 bench.py --workload s2_vocoder --s2-shape $shape --steps 50 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/tp2_${v}_${shape}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/tp2_${v}_${shape}_$i/run_kernel_trace.csv
done
done
done
