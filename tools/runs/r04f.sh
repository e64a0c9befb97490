# Round 4: the stage1 head's plane swizzle (vocoder_x3.hip plane_sw): parity
# tests of the head / vocoder paths, LDS counters and FETCH of the head, a
# pipeline A/B against the previous build; the L2 read rate of time-skewed
# contiguous readers (tools/probe/l2bw.hip ROWS = 3) at the long-form K / V
# size.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_head_comp.py tests/test_gpu_parity.py tests/test_gpu_components_general.py tests/test_gpu_range.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04f_tests.log; [ $rc -eq 0 ] || exit $rc
LDS="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA"
h=gpurun_out/prof_r04f_voc_lds
mkdir -p $h
timeout -s KILL 150 rocprofv3 --pmc $LDS --output-format csv -d $h/lds -o run -- python3 bench.py --steps 4 --warmup 20 --no-cpu-baseline --no-extras > $h/lds.log 2>&1 || exit 1
python3 tools/pmc_summary.py $h --filter x3_head > $h/pmc.txt || exit 1
cat $h/pmc.txt
OLD=m2-tts_amd/csrc/build_old/libm2tts_hip_old.so
for i in 1 2; do for v in new old; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v = old ] && L=$OLD
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f_k_${v}$i -o run -- python3 bench.py --steps 30 --warmup 20 --no-cpu-baseline --no-extras > gpurun_out/r04f_k_${v}$i.json 2> gpurun_out/r04f_k_${v}$i.err || exit 1
  echo "== $v $i $(python3 -c "import json;print(json.loads(open('gpurun_out/r04f_k_${v}$i.json').read().strip().splitlines()[-1])['ms_per_step'])")"
  grep -E "x3_head" gpurun_out/r04f_k_${v}$i/run_kernel_stats.csv | cut -d, -f1-6 | head -3
  rm -f gpurun_out/r04f_k_${v}$i/run_kernel_trace.csv
done; done
for pw in 458752 2097152; do timeout -k 10 120 ./tools/probe/l2bw.bin $pw >> gpurun_out/r04f_l2bw.txt || exit 1; done
cat gpurun_out/r04f_l2bw.txt
