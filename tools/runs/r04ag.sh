# Round 4: first launch at 4 waves per 64-row-tile workgroup as the default
# (fk_nw): tile / device-T / parity tests on the new library; configs[4]
# traces against the 8-wave build alternated; stage2 B=64 with 64-row first
# tiles forced (M2_TFL_FIRST_RB=4) against the default 32-row ones.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
O8=m2-tts_amd/csrc/build_ab/libm2tts_hip_fk8.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_device_T.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ag_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04ag_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in nw4 nw8; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v = nw8 ] && L=$O8
  d=gpurun_out/r04ag_lf_${v}$i
  M2TTS_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $d.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 3 > $d.txt || exit 1
  rm -f $d/run_kernel_trace.csv
  echo "== lf $v $i"; grep -E "span|first_kernel" $d.txt
done; done
for i in 1 2; do for v in rb2 rb4; do
  E=0; [ $v = rb4 ] && E=4
  M2_TFL_FIRST_RB=$E timeout -k 10 300 python3 bench.py --workload s2_b64 --steps 50 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/r04ag_b64_${v}$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r04ag_b64_${v}$i.json').read().strip().splitlines()[-1]);print('s2_b64', '$v', d['ms_per_step'])"
done; done
