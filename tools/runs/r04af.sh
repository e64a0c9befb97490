# Round 4: the first launch at 4 waves per workgroup (-DFK_NW=4: two
# workgroups per CU at 189 VGPRs, so one tile's latency chain overlaps
# another's): tile tests on both libraries, then configs[4] and s2 B=8 kernel
# traces alternated.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
FL=m2-tts_amd/csrc/build_ab/libm2tts_hip_fknw4.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04af_tests_base.log 2>&1
rc=$?; tail -2 gpurun_out/r04af_tests_base.log; [ $rc -eq 0 ] || exit $rc
M2TTS_HIP_LIB=$FL timeout -k 10 400 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_device_T.py -x -q --timeout 120 --timeout-method thread -k "auto or f4 or device or duration or frame" > gpurun_out/r04af_tests_fk.log 2>&1
rc=$?; tail -2 gpurun_out/r04af_tests_fk.log; [ $rc -eq 0 ] || exit $rc
for shape in "128 one 520" "8 one 100"; do
  tag=$(echo $shape | tr ' ' '_')
  for i in 1 2; do for v in base fk; do
    L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v = fk ] && L=$FL
    d=gpurun_out/r04af_${tag}_${v}$i
    M2TTS_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py $shape > $d.log 2>&1 || exit 1
    python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 3 > $d.txt || exit 1
    rm -f $d/run_kernel_trace.csv
    echo "== $tag $v $i"; grep -E "span|first_kernel" $d.txt
  done; done
done
