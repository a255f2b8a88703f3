#!/bin/bash
# round 5: re-check three defaults on the one-stream step (alternated pairs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/r05_defaults_ab.txt
for e in RECBLR_CONV_ROWS RECBLR_DEFER_RESIDUAL RECBLR_TN_FEW; do
  SETTLE=6 bash tools/ab_env.sh "$e=1" "$e=0" 2 >> $OUT/r05_defaults_ab.txt 2>&1 || exit $?
done
cut -c1-50 $OUT/r05_defaults_ab.txt
