# Round 4: XCD-aware head windows (-DX3_HEAD_XCD=1) on the stage2 heads
# (configs[4] chunks, B=8 and B=16 T=2600 vocoder lines): kernel traces and
# the s2 vocoder lines, alternated.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
XL=m2-tts_amd/csrc/build_ab/libm2tts_hip_xcd.so
for i in 1 2; do for v in base xcd; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v = xcd ] && L=$XL
  M2TTS_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04ad_${v}$i -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > gpurun_out/r04ad_${v}$i.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize gpurun_out/r04ad_${v}$i/run_kernel_trace.csv 3 > gpurun_out/r04ad_${v}$i.txt || exit 1
  rm -f gpurun_out/r04ad_${v}$i/run_kernel_trace.csv
  echo "== $v $i"; grep -E "span|x3_head|x3_mid|tailp2" gpurun_out/r04ad_${v}$i.txt
  M2TTS_HIP_LIB=$L timeout -k 10 300 python3 bench.py --workload s2_vocoder --steps 100 --warmup 20 --no-cpu-baseline --no-extras > gpurun_out/r04ad_s2v_${v}$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r04ad_s2v_${v}$i.json').read().strip().splitlines()[-1]);print('s2_vocoder', '$v', d['ms_per_step'], d['config'])"
done; done
