#!/bin/bash
# round 5: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs
# the runtime default: bench alternated, both orders
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
SETTLE=8 bash tools/ab_env.sh "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" 3 > $OUT/r05_ka_ab.txt 2>&1 || exit $?
SETTLE=8 bash tools/ab_env.sh "HIP_FORCE_DEV_KERNARG=0" "HIP_FORCE_DEV_KERNARG=1" 2 >> $OUT/r05_ka_ab.txt 2>&1 || exit $?
cut -c1-56 $OUT/r05_ka_ab.txt
