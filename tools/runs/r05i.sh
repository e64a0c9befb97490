# Round 5: which role of tailr bounds its step - diagnostic builds where the
# front (trd1) or the back (trd2) wave skips its layers (timing only).
set -u
tag=r05i
export TMPDIR=/tmp M2_TAILR=1
mkdir -p gpurun_out
for v in full trd1 trd2; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v != full ] && L=tools/probe/libm2tts_$v.so
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_${v}_1 -o run -- \
      python3 bench.py --workload vocoder --steps 50 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/${tag}_${v}_1.json 2>/dev/null || exit 1
  rm -f gpurun_out/${tag}_${v}_1/run_kernel_trace.csv
done
