# Round 4: (a) where the long-form attention's step time goes: diagnostic
# builds of attention_qsplit2's lean path without one piece each (TFL_DIAG
# bits: 1 global loads, 2 softmax VALU, 4 LDS stores, 8 QK^T MFMAs, 16 PV
# MFMAs, 24 both GEMMs), decoder alone at B=128 T=2600; (b) the XCD-aware
# head windows: head tests, FETCH against batch, kernel-time A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in 0 1 2 4 8 16 24; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $d != 0 ] && L=m2-tts_amd/csrc/build_diag/libm2tts_hip_d$d.so
  M2TTS_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04h_diag_d$d -o run -- python3 tools/probe/dec_time.py 128 2600 6 > gpurun_out/r04h_diag_d$d.log 2>&1 || exit 1
  rm -f gpurun_out/r04h_diag_d$d/run_kernel_trace.csv
  echo "== diag $d $(grep decoder gpurun_out/r04h_diag_d$d.log)"
  python3 - gpurun_out/r04h_diag_d$d/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "layer_kernel" in r["Name"]:
        print("  ", r["Name"].split("(")[0].replace("void m2::tfl::", ""), r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_head_comp.py tests/test_gpu_parity.py tests/test_gpu_device_T.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04h_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04h_tests.log; [ $rc -eq 0 ] || exit $rc
for B in 8 32 128; do
  h=gpurun_out/prof_r04h_head_b$B
  mkdir -p $h
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $h/fetch -o run -- python3 bench.py --batch $B --steps 4 --warmup 20 --no-cpu-baseline --no-extras > $h/fetch.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $h --filter x3_head > $h/pmc.txt || exit 1
  echo "== B=$B"; grep -A2 "x3_head" $h/pmc.txt | head -4
done
NOX=m2-tts_amd/csrc/build_ab/libm2tts_hip_noxcd.so
for i in 1 2; do for v in xcd plain; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v = plain ] && L=$NOX
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04h_k_${v}$i -o run -- python3 bench.py --steps 30 --warmup 20 --no-cpu-baseline --no-extras > gpurun_out/r04h_k_${v}$i.json 2> gpurun_out/r04h_k_${v}$i.err || exit 1
  rm -f gpurun_out/r04h_k_${v}$i/run_kernel_trace.csv
  python3 - gpurun_out/r04h_k_${v}$i/run_kernel_stats.csv $v$i <<'PY'
import csv, sys
print(sys.argv[2], " ".join(f'{r["Name"].split("(")[0].split("::")[-1]} {float(r["AverageNs"]) / 1e3:.2f}us' for r in csv.DictReader(open(sys.argv[1])) if any(k in r["Name"] for k in ("x3_head", "midp", "tailp"))))
PY
done; done
