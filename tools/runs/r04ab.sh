# Round 4: the long-form decoder's first launch compiled for 4 waves per
# SIMD (two workgroups per CU, 128 VGPRs, some spills) against 2: configs[4]
# kernel traces, alternated.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
FK=m2-tts_amd/csrc/build_ab/libm2tts_hip_fk4.so
for i in 1 2; do for v in base fk4; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v = fk4 ] && L=$FK
  M2TTS_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04ab_${v}$i -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > gpurun_out/r04ab_${v}$i.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize gpurun_out/r04ab_${v}$i/run_kernel_trace.csv 3 > gpurun_out/r04ab_${v}$i.txt || exit 1
  rm -f gpurun_out/r04ab_${v}$i/run_kernel_trace.csv
  echo "== $v $i"; grep -E "span|first_kernel" gpurun_out/r04ab_${v}$i.txt
done; done
