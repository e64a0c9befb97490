# Round 5: the rounds-aware stage2 windows (head 16/19/24/27 frames, mid
# 30/33 positions) on the in-tree library: full GPU suite, smoke, then the
# whole bench (no CPU leg) and the configs[4] long-form line for the in-tree
# library and the previous commit's build (build_base), alternated twice.
set -u
tag=r05ac
export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=m2-tts_amd/src/m2amd/libm2tts_hip.so
OLD=m2-tts_amd/csrc/build_base/libm2tts_hip_base.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -n 20 gpurun_out/${tag}_smoke.log; exit 1; }
for i in 1 2; do
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  M2TTS_HIP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/${tag}_bench_${v}_$i.json 2> gpurun_out/${tag}_bench_${v}_$i.err || exit 1
  M2TTS_HIP_LIB=$L timeout -k 10 300 python3 bench.py --workload s2_longform --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/${tag}_lf_${v}_$i.json 2> gpurun_out/${tag}_lf_${v}_$i.err || exit 1
done
done
