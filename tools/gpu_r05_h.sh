#!/bin/bash
# round 5: configs[4] projections dispatched per shape (RECBLR_BF16_GEMM=auto)
# against all-own (1) and all-hipBLASLt (0): tests, then the C5 step alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_gemm_bf16.py tests/test_gpu_bf16.py > $OUT/r05_bfauto_pytest.log 2>&1 || exit $?
tail -1 $OUT/r05_bfauto_pytest.log
for r in 1 2 3; do
  for m in auto 1 0; do
    echo "== $m" >> $OUT/r05_bfauto_c5.txt
    RECBLR_BF16_GEMM=$m timeout -k 10 300 python -u tools/c5_step.py 6 >> $OUT/r05_bfauto_c5.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $OUT/r05_bfauto_c5.txt
