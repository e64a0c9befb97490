# Round 6: PMC passes over the stage2 decoder alone (B=128 T=2600) on
# attention forms 9 and 12 - MFMA busy, VALU, waits, vector-memory cycles.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r06ae_pmc
mkdir -p $out
run() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $out/$n -o run -- python3 tools/probe/dec_time.py 128 2600 2 > $out/$n.log 2>&1; local rc=$?; echo "pass $n rc=$rc"; return $rc; }
for f in 9 12; do
  export M2_TFL_QS2=$f
  run f${f}a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA || exit 1
  run f${f}b SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE || exit 1
  for p in a b; do
    python3 tools/probe/pmc_by_kernel.py $out/f${f}$p/run_counter_collection.csv "layer_kernel<96, false, 1" >> gpurun_out/r06ae_pmc.txt
  done
done
cat gpurun_out/r06ae_pmc.txt
