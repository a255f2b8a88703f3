#!/bin/bash
# round 5: bf16 gate forward variants at configs[4]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 tools/bin/gate_fwd_probe 9 > $OUT/r05_gf_probe.txt 2>&1 || exit $?
cat $OUT/r05_gf_probe.txt
