#!/bin/bash
# round 5: the FeedForward's dU GEMM + activation backward on 256 x 256 tiles
# (ab_dact8.so: 27 spilled registers) vs the shipped 256 x 128: its tests,
# then the bench alternated (ab_gemm.sh: step and per-shape kernel times)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
RECBLR_LIB=datamining_recblr_amd/lib/ab_dact8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_half.py tests/test_gpu_blocks.py -x -q -k "act or feed" --timeout 200 --timeout-method thread > $OUT/r05_d8_pytest.log 2>&1 || exit $?
tail -1 $OUT/r05_d8_pytest.log
SETTLE=8 bash tools/ab_gemm.sh 3 datamining_recblr_amd/lib/ab_dact8.so datamining_recblr_amd/lib/libdmrecblr.so > $OUT/r05_d8_ab.txt 2>&1 || exit $?
cut -c1-80 $OUT/r05_d8_ab.txt
