#!/bin/bash
# round 5: timing ablation — the 256-column NT tiles (NB = 8) with A two
# k-steps ahead through three stages (exponents/bias/flags aliased away:
# results not meaningful) against the shipped one-ahead two stages
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
for b in cur nsa3 cur nsa3; do
  echo "== $b" >> $OUT/r05_nsa3.txt
  timeout -k 10 120 tools/bin/gemm_ab_$b >> $OUT/r05_nsa3.txt 2>&1 || exit $?
done
grep -E "==|total|R=" $OUT/r05_nsa3.txt | grep -v "^ce\|dW"
