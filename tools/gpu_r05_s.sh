#!/bin/bash
# round 5: timing-only ablations of the f16x3 NT GEMM (results not
# meaningful): no MFMAs (operands kept live), no output stores
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
for b in cur nomfma nostore cur nomfma nostore; do
  echo "== $b" >> $OUT/r05_ntabl.txt
  timeout -k 10 120 tools/bin/gemm_ab_$b >> $OUT/r05_ntabl.txt 2>&1 || exit $?
done
grep -E "==|total|R=" $OUT/r05_ntabl.txt | grep -v "^ce\|dW"
