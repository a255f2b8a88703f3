#!/bin/bash
# round 5: the fp32 gate backward (bench shape) in channel passes: two
# waves per SIMD (gate_bf16_probe) and three (gate_probe_occ3: 12 spilled
# registers), against the shipped 8 x 2 layout
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/r05_g32_probe.txt
for r in 1 2; do
  for b in gate_bf16_probe gate_probe_occ3; do
    echo "== $b" >> $OUT/r05_g32_probe.txt
    timeout -k 10 240 tools/bin/$b 7 >> $OUT/r05_g32_probe.txt 2>&1 || exit $?
  done
done
cat $OUT/r05_g32_probe.txt
