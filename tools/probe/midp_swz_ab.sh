# midp ring swizzle: vocoder parity tests, kernel stats of the headline bench
# for the new build and a baseline build (make OBJDIR=build_old ...), and an
# LDS PMC pass of each.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
OLD=m2-tts_amd/csrc/build_old/libm2tts_hip_old.so
NEW=m2-tts_amd/src/m2amd/libm2tts_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "vocoder or pipeline or inference" > gpurun_out/mswz_tests.log 2>&1 || { tail -n 20 gpurun_out/mswz_tests.log; exit 1; }
tail -n 1 gpurun_out/mswz_tests.log
for i in 1 2; do
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mswz_${v}_$i -o run -- \
      python3 bench.py --steps 100 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/mswz_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/mswz_${v}_$i/run_kernel_trace.csv
done
done
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  M2TTS_HIP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/mswz_pmc_$v -o run -- \
      python3 bench.py --steps 4 --warmup 20 --no-cpu-baseline --no-extras > /dev/null 2>&1 || exit 1
done
