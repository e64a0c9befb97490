# Round 4: the base in the tail k-step (head_dim 48 wave-specialised consumers:
# no per-step -m vector build): every tile test, in-process A/B against the
# ping-pong form, long-form PMC pass (VALU:MFMA).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread  > gpurun_out/r04s_tf_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04s_tf_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/env_ab.py M2_TFL_QS2 6,9 s2 128 520 4 2 > gpurun_out/r04s_ab_lf.txt 2>&1 || exit 1
cat gpurun_out/r04s_ab_lf.txt
d=gpurun_out/prof_r04s_lf
mkdir -p $d
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $SQ --output-format csv -d $d/sq -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $d/sq.log 2>&1 || exit 1
python3 tools/pmc_summary.py $d --filter layer_kernel > gpurun_out/r04s_longform_pmc.txt || exit 1
grep -A10 "layer_kernel<96, false, 1" gpurun_out/r04s_longform_pmc.txt | head -11
