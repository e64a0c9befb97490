# PMC passes over the one-launch decoder layers at B=8 T=500.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_tfl
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_tfl/$name -o run -- python3 tools/probe/tfl_run.py 8x500 6 > gpurun_out/pmc_tfl/$name.log 2>&1 || return 1
  python3 tools/probe/pmc_by_kernel.py gpurun_out/pmc_tfl/$name/run_counter_collection.csv layer_kernel > gpurun_out/pmc_tfl/$name.txt
  rm -f gpurun_out/pmc_tfl/$name/run_counter_collection.csv
  cat gpurun_out/pmc_tfl/$name.txt
}
run tcc TCC_HIT_sum TCC_MISS_sum &&
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU &&
run tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum &&
run ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
