#!/bin/bash
# Profile one bench.py configuration on the GPU box with rocprofv3:
# one kernel-trace/stats pass plus separate PMC passes (never combined with
# sys/runtime traces).  Usage: tools/profile_gpu.sh <tag> [bench args...]
# Output: gpurun_out/prof_<tag>/{trace,sq,lds,fetch,write}/...
set -u
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
# enough warm-up for the clocks to settle (bench.py's default), so the kernel
# averages match the bench's own HIP-event timings
BENCH="python3 bench.py --steps 100 --warmup 100 --no-cpu-baseline --no-extras $*"
# PMC passes: counters per dispatch, so a few timed steps are enough
PMCBENCH="python3 bench.py --steps 4 --warmup 20 --no-cpu-baseline --no-extras $*"
run() {  # name, rocprof args...
  local name=$1; shift
  local cmd=$PMCBENCH
  [ "$name" = trace ] && cmd=$BENCH
  timeout -k 10 240 rocprofv3 "$@" --output-format csv -d $out/$name -o run -- $cmd > $out/$name.log 2>&1
  local rc=$?
  # the per-dispatch trace is large; the stats csv is what gets summarised
  rm -f $out/$name/run_kernel_trace.csv
  echo "pass $name rc=$rc"
  return $rc
}
run trace --kernel-trace --stats &&
run sq --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE &&
run lds --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_LDS_UNALIGNED_STALL &&
run fetch --pmc FETCH_SIZE &&
run write --pmc WRITE_SIZE
