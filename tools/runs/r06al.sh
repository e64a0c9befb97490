# Round 6: form 12 with the two-MFMA tail and VALU row sums - full GPU suite,
# configs[4] kernel trace, PMC passes over the decoder, default bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06al_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/r06al_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/r06al_gpu_tests.log
d=gpurun_out/r06al_tr_lf
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $d.log 2>&1 || { tail -n 20 $d.log; exit 1; }
python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 3 > gpurun_out/r06al_tr_lf.txt || exit 1
rm -f $d/run_kernel_trace.csv
cat gpurun_out/r06al_tr_lf.txt
out=gpurun_out/r06al_pmc
mkdir -p $out
run() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $out/$n -o run -- python3 tools/probe/dec_time.py 128 2600 2 > $out/$n.log 2>&1; local rc=$?; echo "pass $n rc=$rc"; return $rc; }
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA || exit 1
run b SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE || exit 1
for p in a b; do python3 tools/probe/pmc_by_kernel.py $out/$p/run_counter_collection.csv "layer_kernel<96, false, 1" >> gpurun_out/r06al_pmc.txt; done
cat gpurun_out/r06al_pmc.txt
timeout -k 10 500 python -u bench.py > gpurun_out/r06al_bench.json 2> gpurun_out/r06al_bench.err || exit 1
grep "ms/step" gpurun_out/r06al_bench.err
