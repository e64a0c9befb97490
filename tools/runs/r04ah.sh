# Round 4: 64-row first-launch tiles (4-wave workgroups) from 8 rounds of
# 16-row tiles (was 16): stage2 B=64 T=500 (configs[3] at N=1) and B=16
# S=520 (configs[4]'s per-GPU share at N=8) against M2_TFL_FIRST_RB=2
# alternated; tile / device-T tests and smoke on the new library.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_device_T.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ah_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04ah_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04ah_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r04ah_smoke.log
for i in 1 2 3; do for v in rb2 auto; do
  E=0; [ $v = rb2 ] && E=2
  M2_TFL_FIRST_RB=$E timeout -k 10 300 python3 bench.py --workload s2_b64 --steps 50 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/r04ah_b64_${v}$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r04ah_b64_${v}$i.json').read().strip().splitlines()[-1]);print('s2_b64', '$v', d['ms_per_step'])"
done; done
for i in 1 2; do for v in rb2 auto; do
  E=0; [ $v = rb2 ] && E=2
  d=gpurun_out/r04ah_b16_${v}$i
  M2_TFL_FIRST_RB=$E timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 16 one 520 > $d.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 3 > $d.txt || exit 1
  rm -f $d/run_kernel_trace.csv
  echo "== b16 $v $i"; grep -E "span|first_kernel" $d.txt
done; done
