# Round 5: wider stage2 head / mid windows (M2_S2_HEAD_TF=32, M2_S2_MID_W=56)
# - bit-identity tests, in-process A/B at the long form and B=64, and the
# configs[4] chunked bench line with both.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_s2_tiles.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05f_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_S2_MID_W unset,56 s2 128 520 4 2 > gpurun_out/r05f_ab_mid_lf.txt 2>&1 || exit 1
cat gpurun_out/r05f_ab_mid_lf.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_S2_HEAD_TF unset,32 s2 128 520 4 2 > gpurun_out/r05f_ab_head_lf.txt 2>&1 || exit 1
cat gpurun_out/r05f_ab_head_lf.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_S2_MID_W unset,56 s2 64 100 6 10 > gpurun_out/r05f_ab_mid_64.txt 2>&1 || exit 1
cat gpurun_out/r05f_ab_mid_64.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_S2_HEAD_TF unset,32 s2 64 100 6 10 > gpurun_out/r05f_ab_head_64.txt 2>&1 || exit 1
cat gpurun_out/r05f_ab_head_64.txt
for i in 1 2; do
  for v in base both; do
    if [ $v = both ]; then export M2_S2_MID_W=56 M2_S2_HEAD_TF=32; else unset M2_S2_MID_W M2_S2_HEAD_TF; fi
    timeout -k 10 300 python3 bench.py --workload s2_longform --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/r05f_lf_${v}$i.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/r05f_lf_${v}$i.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])"
  done
done
