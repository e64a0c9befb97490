# Round 6: stage1 mid with the LDS-DMA loader (MIDP_DMA=1, the new build)
# against the register loader (build_base, MIDP_DMA=0): tail / range /
# stress / streaming / parity tests on the new build, then the headline's
# kernel stats and the vocoder bench line, alternated twice.
set -u
tag=r06u
export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=m2-tts_amd/src/m2amd/libm2tts_hip.so
OLD=m2-tts_amd/csrc/build_base/libm2tts_hip_base.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_tailp.py tests/test_gpu_head_comp.py tests/test_gpu_range.py tests/test_gpu_stress.py tests/test_gpu_sharding_streaming.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
for i in 1 2; do
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  d=gpurun_out/${tag}_${v}_$i
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 bench.py --steps 100 --warmup 100 --no-cpu-baseline --no-extras > $d.json 2>/dev/null || exit 1
  rm -f $d/run_kernel_trace.csv
  grep -E "midp|tailp" $d/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/$v $i /" | cut -c1-60,200-
  M2TTS_HIP_LIB=$L timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-extras > ${d}_bench.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('${d}_bench.json').read().strip().splitlines()[-1]); print('$v $i', d['ms_per_step'], d['roofline']['avg_kernel_ms'])"
done
done
