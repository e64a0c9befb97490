# Round 4 closing record (final defaults): full GPU suite, smoke, default and driver-form
# bench, the headline's kernel trace + PMC passes (traffic.json refreshed
# from them), the long-form decoder layer's PMC pass (VALU:MFMA) and kernel
# trace on the default forms, the B=8 share's kernel trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04x_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04x_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04x_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/r04x_smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/r04x_bench.json 2> gpurun_out/r04x_bench.err || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04x_bench_driver.json 2> gpurun_out/r04x_bench_driver.err || exit 1
python3 - <<'PY'
import json
for f in ("gpurun_out/r04x_bench.json", "gpurun_out/r04x_bench_driver.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"], {k: d[k]["ms_per_step"] for k in d if isinstance(d[k], dict) and "ms_per_step" in d[k]})
PY
bash tools/profile_gpu.sh r04x || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_r04x --traffic gpurun_out/r04x_traffic.json > gpurun_out/r04x_pmc.txt || exit 1
python3 tools/prof_summary.py gpurun_out/prof_r04x > gpurun_out/r04x_prof.txt 2>&1 || true
cat gpurun_out/r04x_traffic.json
d=gpurun_out/prof_r04x_lf
mkdir -p $d
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $SQ --output-format csv -d $d/sq -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $d/sq.log 2>&1 || exit 1
python3 tools/pmc_summary.py $d --filter layer_kernel > gpurun_out/r04x_longform_pmc.txt || exit 1
grep -A12 "layer_kernel<96, false, 1" gpurun_out/r04x_longform_pmc.txt | head -13
for w in "128 one 520" "8 dev 100"; do
  tag=$(echo $w | tr ' ' _)
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04x_tr_$tag -o run -- python3 tools/probe/s2_small_trace.py $w > gpurun_out/r04x_tr_$tag.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize gpurun_out/r04x_tr_$tag/run_kernel_trace.csv $([ "$tag" = "128_one_520" ] && echo 3 || echo 20) > gpurun_out/r04x_tr_$tag.txt || exit 1
  rm -f gpurun_out/r04x_tr_$tag/run_kernel_trace.csv
  head -16 gpurun_out/r04x_tr_$tag.txt
done
