# Round 5: the stage2 pipelined tail with a run-time strip length (any length
# 8-256 chosen by the rounds x steps model): its tests, then kernel stats at
# 8x500 / 16x2600 and the long-form chunked line, against the round's
# previous library (m2-tts_amd/csrc/build_old, instantiated lengths), alternated.
set -u
tag=r05t
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tailp2.py tests/test_gpu_sharding_streaming.py tests/test_gpu_range.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 20 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
OLD=m2-tts_amd/csrc/build_old/libm2tts_hip_old.so
NEW=m2-tts_amd/src/m2amd/libm2tts_hip.so
for i in 1 2; do
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  for sh in 8x500 16x2600; do
    M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_${sh}_${v}_$i -o run -- \
        python3 bench.py --workload s2_vocoder --s2-shape $sh --steps 30 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/${tag}_${sh}_${v}_$i.json 2>/dev/null || exit 1
    rm -f gpurun_out/${tag}_${sh}_${v}_$i/run_kernel_trace.csv
  done
  M2TTS_HIP_LIB=$L timeout -k 10 300 python3 bench.py --workload s2_longform --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${tag}_lf_${v}_$i.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_lf_${v}_$i.json').read().strip().splitlines()[-1]); print('lf $v', d['ms_per_step'])"
done
done
