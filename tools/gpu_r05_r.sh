#!/bin/bash
# round 5: gate-scan backward lane layout A/B: Q time chunks x TC steps per
# lane (Q = 8 shipped; 4 and 16): parity tests on each, then the bench's
# gate-scan / conv fractions alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
L=datamining_recblr_amd/lib
mkdir -p $OUT
for v in gq4 gq16; do
  RECBLR_LIB=$L/ab_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_scale.py -k "gate or grl or scan" > $OUT/r05_gq_pytest_$v.log 2>&1 || exit $?
  tail -1 $OUT/r05_gq_pytest_$v.log
done
SETTLE=5 timeout -k 10 1000 bash tools/ab_multi.sh 2 $L/libdmrecblr.so $L/ab_gq4.so $L/ab_gq16.so > $OUT/r05_gq_ab.txt 2>&1 || exit $?
cat $OUT/r05_gq_ab.txt
