#!/bin/bash
# SQ counters of the fused GatedRecurrentLayer kernels (tools/grlbench.hip):
# wave cycles split into waiting / issue-stalled / active, VALU / LDS / MFMA
# issue.  One counter group per pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM --output-format csv -d $OUT/pmc_grl1 -o run -- tools/bin/grlbench_p0 2048 200 3 > $OUT/pmc_grl1.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA --output-format csv -d $OUT/pmc_grl2 -o run -- tools/bin/grlbench_p0 2048 200 3 > $OUT/pmc_grl2.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM --output-format csv -d $OUT/pmc_grl3 -o run -- tools/bin/grlbench_p0 2048 200 3 > $OUT/pmc_grl3.log 2>&1 || exit $?
