#!/bin/bash
# SQ counters of the f16 split GEMM (tools/bin/gbh_base: all projection shapes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
BIN=${1:-tools/bin/gemmbench_h_nb4}
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $OUT/pmc_gh1 -o run -- $BIN > $OUT/pmc_gh1.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/pmc_gh2 -o run -- $BIN > $OUT/pmc_gh2.log 2>&1 || exit $?
find $OUT/pmc_gh1 $OUT/pmc_gh2 -name "*counter_collection*"
