# Generic A/B of the in-tree library against a baseline build
# (make -C m2-tts_amd/csrc OBJDIR=build_old OUT=build_old/libm2tts_hip_old.so
# from the previous commit): GPU parity file(s) $TESTS, then kernel stats of
# bench.py --workload $WL for both builds, alternated twice.
#   TESTS="tests/test_gpu_parity.py" WL=pipeline bash tools/probe/lib_ab.sh <tag>
set -u
tag=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
OLD=m2-tts_amd/csrc/build_old/libm2tts_hip_old.so
NEW=m2-tts_amd/src/m2amd/libm2tts_hip.so
WL=${WL:-pipeline}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 20 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
for i in 1 2; do
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_${v}_$i -o run -- \
      python3 bench.py --workload $WL --steps 100 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/${tag}_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/${tag}_${v}_$i/run_kernel_trace.csv
done
done
