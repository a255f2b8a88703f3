#!/bin/bash
# round 5: the embedding backward's plan (counting sort of the ids) on its
# side stream during the forward (RECBLR_EMB_SIDE=1) vs inline on the current
# stream (=0): tests with it inline, then the bench alternated both orders
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
RECBLR_EMB_SIDE=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_blocks.py tests/test_gpu_timed_step.py -x -q --timeout 200 --timeout-method thread > $OUT/r05_es_pytest.log 2>&1 || exit $?
tail -1 $OUT/r05_es_pytest.log
SETTLE=8 bash tools/ab_env.sh "RECBLR_EMB_SIDE=1" "RECBLR_EMB_SIDE=0" 3 > $OUT/r05_es_ab.txt 2>&1 || exit $?
SETTLE=8 bash tools/ab_env.sh "RECBLR_EMB_SIDE=0" "RECBLR_EMB_SIDE=1" 2 >> $OUT/r05_es_ab.txt 2>&1 || exit $?
cut -c1-50 $OUT/r05_es_ab.txt
