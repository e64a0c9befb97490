# Round 4: HBM bytes of the long-form first launch (frame expansion -> LN1 ->
# QKV, first_kernel<96, 2, ...>) and of the encoder / decoder layer launches
# at configs[4] (s2 B=128 S=520, one-call inference): FETCH_SIZE and
# WRITE_SIZE passes, each its own run.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
h=gpurun_out/prof_r04ae_lf
mkdir -p $h
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $h/fetch -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $h/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $h/write -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $h/write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM --output-format csv -d $h/sq -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $h/sq.log 2>&1 || exit 1
for f in first_kernel layer_kernel duration x3_head; do
  echo "== $f"; python3 tools/pmc_summary.py $h --filter $f || exit 1
done > gpurun_out/r04ae_pmc.txt
cat gpurun_out/r04ae_pmc.txt
