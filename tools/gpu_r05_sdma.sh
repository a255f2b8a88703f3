#!/bin/bash
# round 5: the packed layout's per-step host -> device copy through the SDMA
# engine (default) vs a blit kernel on the compute queue (HSA_ENABLE_SDMA=0):
# bench alternated, both orders
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
SETTLE=8 bash tools/ab_env.sh "HSA_ENABLE_SDMA=1" "HSA_ENABLE_SDMA=0" 3 > $OUT/r05_sdma_ab.txt 2>&1 || exit $?
SETTLE=8 bash tools/ab_env.sh "HSA_ENABLE_SDMA=0" "HSA_ENABLE_SDMA=1" 2 >> $OUT/r05_sdma_ab.txt 2>&1 || exit $?
cut -c1-50 $OUT/r05_sdma_ab.txt
