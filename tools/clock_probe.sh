#!/bin/bash
# Box diagnostics for the gate backward's box-to-box spread: clocks/power as
# reported, kbench's gate-backward lines, and one PMC pass whose
# GRBM_GUI_ACTIVE / kernel duration gives the effective shader clock.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
(rocm-smi --showclocks --showpower --showperflevel --showmaxpower 2>&1 || true) > $OUT/smi.log
timeout -k 10 120 tools/bin/kbench 2048 200 256 10 2 > $OUT/kbench_gate.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVES --kernel-trace \
  --output-format csv -d $OUT/pmc_clk -o run -- tools/bin/kbench 2048 200 256 3 2 > $OUT/pmc_clk.log 2>&1 || exit $?
(rocm-smi --showclocks 2>&1 || true) >> $OUT/smi.log
