#!/bin/bash
# round 5: order bias of tools/ab_env.sh — an A/A pair (same setting twice)
# and the copy-ahead A/B with the order reversed (old setting first)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
SETTLE=8 bash tools/ab_env.sh "RECBLR_COPY_AHEAD=0" "RECBLR_COPY_AHEAD=0" 2 > $OUT/r05_ord_aa.txt 2>&1 || exit $?
cut -c1-50 $OUT/r05_ord_aa.txt
SETTLE=8 bash tools/ab_env.sh "RECBLR_COPY_AHEAD=0" "RECBLR_COPY_AHEAD=1" 3 > $OUT/r05_ord_ab.txt 2>&1 || exit $?
cut -c1-50 $OUT/r05_ord_ab.txt
