set -u
for v in NOSPLIT NOEXP NOPV NOQK; do
  M2TTS_HIP_LIB=tools/probe/libm2_$v.so timeout -k 10 100 python tools/probe/att_bench.py --iters 100 > gpurun_out/att_$v.json 2>/dev/null || exit 1
done
