# Round 3 A/B: attention_qsplit2 without runtime array indexing (in-process, M2_TFL_QS2), and (library builds,
# alternated, M2_TFL_QS2=0 in both) tile-independent loads issued before the work-queue claim in the one-launch layers.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
OLD=m2-tts_amd/csrc/build_old/libm2tts_hip_old.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_device_T.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ad_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03ad_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r03ad_ab.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 0,1 s1 32 100 8 40 >> gpurun_out/r03ad_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 0,1 s2 64 100 6 20 >> gpurun_out/r03ad_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 0,1 s2 16 520 5 4 >> gpurun_out/r03ad_ab.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r03ad_ab.txt | cut -c1-110
export M2_TFL_QS2=0
for i in 1 2; do
for v in new old; do
for B in 8 64; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v = old ] && L=$OLD
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ad_$v -o run -- python3 tools/probe/s2_small_trace.py $B dev > gpurun_out/ad_$v.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize gpurun_out/ad_$v/run_kernel_trace.csv > gpurun_out/ad_${v}_${B}_$i.txt || exit 1
  rm -f gpurun_out/ad_$v/run_kernel_trace.csv
  echo "$v B=$B run $i: $(head -1 gpurun_out/ad_${v}_${B}_$i.txt)" | tee -a gpurun_out/r03ad_ab.txt
done
done
done
cat gpurun_out/ad_new_8_2.txt gpurun_out/ad_old_8_2.txt
