#!/bin/bash
# round 5: HIP_FORCE_DEV_KERNARG=1 vs the runtime default (variable unset)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
SETTLE=8 bash tools/ab_env.sh "HIP_FORCE_DEV_KERNARG=1" "RECBLR_NOTHING=1" 3 > $OUT/r05_ka2_ab.txt 2>&1 || exit $?
SETTLE=8 bash tools/ab_env.sh "RECBLR_NOTHING=1" "HIP_FORCE_DEV_KERNARG=1" 2 >> $OUT/r05_ka2_ab.txt 2>&1 || exit $?
cut -c1-56 $OUT/r05_ka2_ab.txt
