#!/bin/bash
# round 5: conv backward chunk/step variants (bf16 configs[4], fp32 bench shape)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 240 tools/bin/conv_bwd_probe 7 > $OUT/r05_cb_probe.txt 2>&1 || exit $?
cat $OUT/r05_cb_probe.txt
