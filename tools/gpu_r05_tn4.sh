#!/bin/bash
# round 5: the bf16 weight-gradient kernel with one wave per SIMD (4 waves of
# 128 x 128, 32-row k-steps, three in flight; ab_tn4.so) vs the shipped one
# (8 waves of 64 x 128, 64-row k-steps, one in flight): its GPU tests, then
# the per-shape probe alternated (RECBLR_BF16_GEMM=1: ours on every shape)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
RECBLR_LIB=datamining_recblr_amd/lib/ab_tn4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_bf16.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > $OUT/r05_tn4_pytest.log 2>&1 || exit $?
tail -1 $OUT/r05_tn4_pytest.log
: > $OUT/r05_tn4_shapes.txt
for r in 1 2; do
  for lib in datamining_recblr_amd/lib/ab_tn4.so datamining_recblr_amd/lib/libdmrecblr.so; do
    echo "== $(basename $lib)" >> $OUT/r05_tn4_shapes.txt
    RECBLR_BF16_GEMM=1 RECBLR_LIB=$lib timeout -k 10 300 python tools/bf16_gemm_probe.py >> $OUT/r05_tn4_shapes.txt 2>&1 || exit $?
  done
done
grep -E "==|TN" $OUT/r05_tn4_shapes.txt
