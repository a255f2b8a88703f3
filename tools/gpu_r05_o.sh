#!/bin/bash
# round 5: bf16 weight gradient with 48-row k-steps, two in flight (product)
# against 64-row steps, one in flight (ab_tn64): tests, TN shapes (all on our
# kernels), C5 step in the all-own mode
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
L=datamining_recblr_amd/lib
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_gemm_bf16.py tests/test_gpu_bf16.py > $OUT/r05_tn48_pytest.log 2>&1 || exit $?
tail -1 $OUT/r05_tn48_pytest.log
for lib in libdmrecblr.so ab_tn64.so libdmrecblr.so ab_tn64.so; do
  echo "== $lib" >> $OUT/r05_tn48_shapes.txt
  RECBLR_BF16_GEMM=1 RECBLR_LIB=$L/$lib timeout -k 10 300 python -u tools/bf16_gemm_probe.py >> $OUT/r05_tn48_shapes.txt 2>&1 || exit $?
done
grep -E "==|TN" $OUT/r05_tn48_shapes.txt
for lib in libdmrecblr.so ab_tn64.so libdmrecblr.so ab_tn64.so; do
  echo "== $lib" >> $OUT/r05_tn48_c5.txt
  RECBLR_LIB=$L/$lib RECBLR_BF16_GEMM=1 timeout -k 10 300 python -u tools/c5_step.py 6 >> $OUT/r05_tn48_c5.txt 2>&1 || exit $?
done
grep -v amdgpu.ids $OUT/r05_tn48_c5.txt
