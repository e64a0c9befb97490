# Strip-length sweep of the pipelined stage1 mid / tail at B=32 T=500
# (M2_MIDP_NCH, M2_TAILP_NCH), kernel stats, alternated on one box.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
for v in d t32 t48 m8 m32; do
  unset M2_TAILP_NCH M2_MIDP_NCH
  case $v in t32) export M2_TAILP_NCH=32;; t48) export M2_TAILP_NCH=48;; m8) export M2_MIDP_NCH=8;; m32) export M2_MIDP_NCH=32;; esac
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nch_${v}_$i -o run -- \
      python3 bench.py --steps 100 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/nch_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/nch_${v}_$i/run_kernel_trace.csv
done
done
