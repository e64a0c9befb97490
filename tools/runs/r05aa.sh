# Round 5: stage2 vocoder kernel stats at the long-form chunk shapes (16 x 262:
# configs[4]'s per-GPU share at N=8, 128 x 262 at N=1) and 64 x 500.
set -u
tag=r05aa
export TMPDIR=/tmp
mkdir -p gpurun_out
for sh in 16x262 128x262 64x500; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_${sh}_base_1 -o run -- \
      python3 bench.py --workload s2_vocoder --s2-shape $sh --steps 30 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/${tag}_${sh}_base_1.json 2>/dev/null || exit 1
  rm -f gpurun_out/${tag}_${sh}_base_1/run_kernel_trace.csv
done
