#!/bin/bash
# round 5: configs[4] bf16 gate backward in channel-pass variants (timing +
# checksums against the shipped variant)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 240 tools/bin/gate_bf16_probe 1024 2048 512 7 > $OUT/r05_gb_probe.txt 2>&1 || exit $?
cat $OUT/r05_gb_probe.txt
