#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, as gfx950
# requires): HBM FETCH_SIZE, WRITE_SIZE and the MFMA busy/FLOP counters.
# Summaries: tools/pmc_traffic.py, tools/pmc_mfma.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
ARGS="--steps 3 --warmup 1 --settle-seconds 0 --no-cpu-baseline --no-full-tail --no-c5"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run \
  -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run \
  -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 --output-format csv \
  -d $OUT/pmc_mfma -o run -- python3 bench.py $ARGS > $OUT/pmc_mfma.log 2>&1 || exit $?
python tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write > $OUT/pmc_traffic.json &&
python tools/pmc_mfma.py $OUT/pmc_mfma > $OUT/pmc_mfma.json
