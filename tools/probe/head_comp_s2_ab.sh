# Stage2 head: composed input_conv o ConvT1 (generic item path) vs the two
# layers (M2_HEAD_INCONV=1), stage2 vocoder at B=8 T=500 and B=16 T=2600,
# arms alternated on one box.  Table: python tools/probe/ab_table.py h2 head
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for shape in 8x500 16x2600; do
for i in 1 2; do
for v in comp inconv; do
  unset M2_HEAD_INCONV
  if [ $v = inconv ]; then export M2_HEAD_INCONV=1; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/h2_${shape}_${v}_$i -o run -- \
      python3 bench.py --workload s2_vocoder --s2-shape $shape --steps 50 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/h2_${shape}_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/h2_${shape}_${v}_$i/run_kernel_trace.csv
done
done
done
