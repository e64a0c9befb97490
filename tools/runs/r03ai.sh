# Round 3: PMC passes over the long-form stage2 step (B=128, S=520 -> T=2600; decoder attention inside the
# one-launch layers): waits, MFMA vs VALU issue, LDS, HBM bytes per kernel (separate --pmc passes, no traces).
set -u
export TMPDIR=/tmp
out=gpurun_out/prof_r03lf
mkdir -p $out
CMD="python3 tools/probe/s2_small_trace.py 128 one 520"
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d $out/$name -o run -- $CMD > $out/$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES &&
pass valu SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE &&
pass lds SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_LDS_UNALIGNED_STALL &&
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE || exit 1
python3 tools/pmc_summary.py $out --json $out/pmc.json > $out/pmc.txt || exit 1
find $out -name "*counter_collection.csv" -delete
cat $out/pmc.txt | head -60
