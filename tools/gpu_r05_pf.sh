#!/bin/bash
# round 5: the f16 weight images refreshed on a side stream at the step's
# start (RECBLR_SPLIT_PREFETCH=1, new default) vs in front of the first
# projection (=0): the multi-step GPU tests, then the bench alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_optim.py tests/test_gpu_timed_step.py tests/test_gpu_e2e.py tests/test_gpu_ddp.py tests/test_gpu_gemm_half.py tests/test_gpu_blocks.py -x -q --timeout 200 --timeout-method thread > $OUT/r05_pf_pytest.log 2>&1 || exit $?
tail -1 $OUT/r05_pf_pytest.log
SETTLE=8 bash tools/ab_env.sh "RECBLR_SPLIT_PREFETCH=1" "RECBLR_SPLIT_PREFETCH=0" 3 > $OUT/r05_pf_ab.txt 2>&1 || exit $?
cat $OUT/r05_pf_ab.txt
