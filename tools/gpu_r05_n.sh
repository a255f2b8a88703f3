#!/bin/bash
# round 5: register-A NT GEMM with A two k-steps ahead (gemm_ab_areg2)
# against the LDS-DMA A stage (gemm_ab_cur); checksums must agree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
for b in cur areg2 cur areg2; do
  echo "== $b" >> $OUT/r05_areg2_ab.txt
  timeout -k 10 120 tools/bin/gemm_ab_$b >> $OUT/r05_areg2_ab.txt 2>&1 || exit $?
done
grep -E "==|total|in.fwd|gates.fwd" $OUT/r05_areg2_ab.txt
