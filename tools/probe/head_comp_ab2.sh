# Head A/B, order swapped (two-layer head first), three rounds; bench only.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
for v in inconv comp; do
  unset M2_HEAD_INCONV
  if [ $v = inconv ]; then export M2_HEAD_INCONV=1; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hd_${v}_$i -o run -- \
      python3 bench.py --steps 200 --warmup 200 --no-cpu-baseline --no-extras > gpurun_out/hd_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/hd_${v}_$i/run_kernel_trace.csv
done
done
