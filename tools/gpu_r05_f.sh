#!/bin/bash
# round 5: f16x3 NT GEMM timing ablation: the 32x32x16 MFMAs replaced by two
# 16x16x32 ones each (same flops and cycles, results not meaningful) — does
# the MFMA shape change the clock the projection GEMMs hold?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
for b in cur mf16 cur mf16; do
  echo "== $b" >> $OUT/r05_mf16_f16_ab.txt
  timeout -k 10 120 tools/bin/gemm_ab_$b >> $OUT/r05_mf16_f16_ab.txt 2>&1 || exit $?
done
grep -E "==|total" $OUT/r05_mf16_f16_ab.txt
