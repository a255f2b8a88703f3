#!/bin/bash
# round 5: effective shader clock per kernel in the bench step
# (GRBM_GUI_ACTIVE with the kernel trace, one counter pass)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
ARGS="--steps 6 --warmup 2 --settle-seconds 0 --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc_clk -o run \
  -- python3 bench.py $ARGS > $OUT/pmc_clk.log 2>&1 || exit $?
python tools/pmc_clock.py $OUT/pmc_clk > $OUT/r05_pmc_clock.txt 2>&1
rm -rf $OUT/pmc_clk
cat $OUT/r05_pmc_clock.txt
