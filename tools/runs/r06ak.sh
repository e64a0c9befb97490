# Round 6: forms 12 / 18 (row sums by VALU) again, more rounds, plus per-kernel
# decoder-layer times from kernel traces of each.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/probe/env_ab.py M2_TFL_QS2 12,18 s2 128 520 10 2 > gpurun_out/r06ak_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r06ak_ab_lf.txt
for f in 12 18 12 18; do
  export M2_TFL_QS2=$f
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06ak_dec_$f -o run -- python3 tools/probe/dec_time.py 128 2600 10 >> gpurun_out/r06ak_dec.txt 2>&1 || exit 1
  grep "layer_kernel" gpurun_out/r06ak_dec_$f/run_kernel_stats.csv | cut -d, -f1-5 >> gpurun_out/r06ak_dec.txt
  rm -f gpurun_out/r06ak_dec_$f/run_kernel_trace.csv
done
cat gpurun_out/r06ak_dec.txt
