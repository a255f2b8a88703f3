#!/bin/bash
# round 5: timing ablations of the f16x3 NT GEMM's data path (results not
# meaningful): no B (weight) DMAs, no A DMAs, no MFMAs, no output stores
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
for b in cur nobdma noadma nomfma nostore cur nobdma noadma; do
  echo "== $b" >> $OUT/r05_ntabl2.txt
  timeout -k 10 120 tools/bin/gemm_ab_$b >> $OUT/r05_ntabl2.txt 2>&1 || exit $?
done
grep -E "==|^total" $OUT/r05_ntabl2.txt
