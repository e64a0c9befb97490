# Round 4: PMC passes of the long-form decoder layer (lean softmax, VALU:MFMA)
# and the stage1 head's FETCH_SIZE against the batch (weights per XCD vs mel
# bytes), LDS counters of the stage1 vocoder kernels.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
LDS="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA"
d=gpurun_out/prof_r04c_lf
mkdir -p $d
timeout -s KILL 150 rocprofv3 --pmc $SQ --output-format csv -d $d/sq -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $d/sq.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc $LDS --output-format csv -d $d/lds -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $d/lds.log 2>&1 || exit 1
python3 tools/pmc_summary.py $d --filter layer_kernel --json $d/pmc.json > $d/pmc.txt || exit 1
cat $d/pmc.txt
for B in 8 32 128; do
  h=gpurun_out/prof_r04c_head_b$B
  mkdir -p $h
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $h/fetch -o run -- python3 bench.py --batch $B --steps 4 --warmup 20 --no-cpu-baseline --no-extras > $h/fetch.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $h --filter x3_head > $h/pmc.txt || exit 1
  echo "== B=$B"; grep -A2 "x3_head" $h/pmc.txt | head -4
done
h=gpurun_out/prof_r04c_voc_lds
mkdir -p $h
timeout -s KILL 150 rocprofv3 --pmc $LDS --output-format csv -d $h/lds -o run -- python3 bench.py --steps 4 --warmup 20 --no-cpu-baseline --no-extras > $h/lds.log 2>&1 || exit 1
python3 tools/pmc_summary.py $h > $h/pmc.txt || exit 1
cat $h/pmc.txt | head -60
