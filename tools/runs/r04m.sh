# Round 4: the wave-specialised attention with interleaved matrix / vector
# regions (8), LDS-DMA staging (9, 10 with 8) against the plain wave-specialised form (7): tile
# tests, in-process A/Bs, decoder-alone kernel times.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread -k "4q7 or 4q8 or 4q9 or 4q10" > gpurun_out/r04m_tf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04m_tf_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 7,8,9,10 s2 128 520 4 2 > gpurun_out/r04m_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r04m_ab_lf.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 7,8,9,10 s2 16 520 6 4 > gpurun_out/r04m_ab_16.txt 2>&1 || exit 1
cat gpurun_out/r04m_ab_16.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 7,8,9,10 s2 64 100 6 10 > gpurun_out/r04m_ab_64.txt 2>&1 || exit 1
cat gpurun_out/r04m_ab_64.txt
for v in 10 9 8 7; do
  M2_TFL_QS2=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04m_dec_q$v -o run -- python3 tools/probe/dec_time.py 128 2600 6 > gpurun_out/r04m_dec_q$v.log 2>&1 || exit 1
  rm -f gpurun_out/r04m_dec_q$v/run_kernel_trace.csv
  python3 - gpurun_out/r04m_dec_q$v/run_kernel_stats.csv "q$v $(grep decoder gpurun_out/r04m_dec_q$v.log)" <<'PY'
import csv, sys
print(sys.argv[2], " | ".join(f'{r["Name"].split("(")[0].replace("void m2::tfl::", "")} {float(r["AverageNs"]) / 1e3:.1f}us' for r in csv.DictReader(open(sys.argv[1])) if "layer_kernel" in r["Name"]))
PY
done
