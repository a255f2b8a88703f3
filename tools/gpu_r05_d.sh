#!/bin/bash
# round 5: bf16 NT with swapped MFMA operands + permlane32 swaps -> 16-B
# stores (ab_bfswap.so) against the shipped kernel: tests on the variant,
# per-shape timings of both, configs[4] step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
L=datamining_recblr_amd/lib
mkdir -p $OUT
RECBLR_LIB=$L/ab_bfswap.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_gemm_bf16.py > $OUT/r05_bfswap_pytest.log 2>&1 || exit $?
tail -2 $OUT/r05_bfswap_pytest.log
for lib in libdmrecblr.so ab_bfswap.so libdmrecblr.so ab_bfswap.so; do
  echo "== $lib" >> $OUT/r05_bfswap_shapes.txt
  RECBLR_LIB=$L/$lib timeout -k 10 300 python -u tools/bf16_gemm_probe.py >> $OUT/r05_bfswap_shapes.txt 2>&1 || exit $?
done
for lib in libdmrecblr.so ab_bfswap.so; do
  echo "== $lib" >> $OUT/r05_bfswap_c5.txt
  RECBLR_LIB=$L/$lib RECBLR_BF16_GEMM=1 timeout -k 10 300 python -u tools/c5_step.py 4 >> $OUT/r05_bfswap_c5.txt 2>&1 || exit $?
done
RECBLR_BF16_GEMM=0 timeout -k 10 300 python -u tools/c5_step.py 4 >> $OUT/r05_bfswap_c5.txt 2>&1
cat $OUT/r05_bfswap_c5.txt | tail -12
