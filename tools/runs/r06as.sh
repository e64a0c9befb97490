# Round 6 closing record after the key-quarter attention: full GPU suite, smoke,
# driver-form and default benches, the headline kernel stats + PMC passes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06as_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/r06as_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/r06as_gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06as_smoke.log 2>&1 || { tail -n 20 gpurun_out/r06as_smoke.log; exit 1; }
tail -n 1 gpurun_out/r06as_smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06as_bench_driver.json 2> gpurun_out/r06as_bench_driver.err || exit 1
grep "ms/step" gpurun_out/r06as_bench_driver.err
timeout -k 10 500 python -u bench.py > gpurun_out/r06as_bench.json 2> gpurun_out/r06as_bench.err || exit 1
grep "ms/step" gpurun_out/r06as_bench.err
bash tools/profile_gpu.sh r06as || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_r06as --traffic gpurun_out/r06as_traffic.json > gpurun_out/r06as_pmc.txt || exit 1
python3 tools/prof_summary.py gpurun_out/prof_r06as > gpurun_out/r06as_prof.txt 2>&1 || true
cat gpurun_out/r06as_traffic.json
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06as_bench_n2.json 2> gpurun_out/r06as_bench_n2.err || { tail -n 20 gpurun_out/r06as_bench_n2.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06as_bench_n2.json").read().strip().splitlines()[-1])
print({k: (d[k]["ms_per_step"], d[k].get("parity", {}).get("bitwise_equal")) for k in d if isinstance(d[k], dict) and "parity" in d[k]})
PY
d=gpurun_out/r06as_tr_lf
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $d.log 2>&1 || { tail -n 20 $d.log; exit 1; }
python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 3 > gpurun_out/r06as_tr_lf.txt || exit 1
rm -f $d/run_kernel_trace.csv
cat gpurun_out/r06as_tr_lf.txt
