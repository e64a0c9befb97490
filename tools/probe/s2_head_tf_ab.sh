# Stage2 composed head: 24-frame windows on large grids (default) vs always
# 16 (M2_S2_HEAD_TF16=1): tests, then stage2 vocoder kernel stats at 16x2600
# and 64x500 (8x500 keeps 16 either way), alternated on one box.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_head_comp.py tests/test_gpu_parity.py tests/test_gpu_sharding_streaming.py tests/test_gpu_tailp2.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tf_tests.log 2>&1 || { tail -n 30 gpurun_out/tf_tests.log; exit 1; }
tail -n 1 gpurun_out/tf_tests.log
for shape in 16x2600 64x500; do
for i in 1 2; do
for v in w24 t16; do
  unset M2_S2_HEAD_TF16
  if [ $v = t16 ]; then export M2_S2_HEAD_TF16=1; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tf_${shape}_${v}_$i -o run -- \
      python3 bench.py --workload s2_vocoder --s2-shape $shape --steps 50 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/tf_${shape}_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/tf_${shape}_${v}_$i/run_kernel_trace.csv
done
done
done
