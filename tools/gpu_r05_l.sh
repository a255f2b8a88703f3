#!/bin/bash
# round 5: the f16x3 NT GEMM with its A rows loaded straight into registers
# (one k-step ahead, no LDS stage; -DHN_A_REG=1) against the LDS-DMA A stage
# (the shipped form, and the same source with HN_A_REG=0): eight encoder
# shapes, checksums must agree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
for b in cur areg1 areg0 cur areg1 areg0; do
  echo "== $b" >> $OUT/r05_areg_ab.txt
  timeout -k 10 120 tools/bin/gemm_ab_$b >> $OUT/r05_areg_ab.txt 2>&1 || exit $?
done
grep -E "==|total|in.fwd|gates.fwd" $OUT/r05_areg_ab.txt
