#!/bin/bash
# round 5: torch's caching allocator with expandable segments vs the default
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
SETTLE=8 bash tools/ab_env.sh "PYTORCH_HIP_ALLOC_CONF=expandable_segments:True" "RECBLR_NOTHING=1" 3 > $OUT/r05_alloc_ab.txt 2>&1 || exit $?
SETTLE=8 bash tools/ab_env.sh "RECBLR_NOTHING=1" "PYTORCH_HIP_ALLOC_CONF=expandable_segments:True" 2 >> $OUT/r05_alloc_ab.txt 2>&1 || exit $?
cut -c1-70 $OUT/r05_alloc_ab.txt
