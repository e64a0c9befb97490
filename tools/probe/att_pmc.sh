#!/bin/bash
# PMC passes over the attention microbenchmark (one shape); separate passes, kernel-trace only.
set -u
export TMPDIR=/tmp
out=gpurun_out/att_pmc
mkdir -p $out
SH=${1:-128x2600x96}
run() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $out/$n -o run -- python3 tools/probe/att_bench.py --iters 10 --shapes $SH > $out/$n.log 2>&1; echo "pass $n rc=$?"; }
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA &&
run b SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM &&
run c SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_INSTS_BRANCH
