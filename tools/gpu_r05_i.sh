#!/bin/bash
# round 5: bf16 TN (weight gradient) on 16x16x32 MFMA blocks (product build)
# against the 32x32x16 kernel (ab_tn32): tests, per-shape timings (all
# shapes on our kernels), C5 step in the per-shape and all-own modes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
L=datamining_recblr_amd/lib
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_gemm_bf16.py tests/test_gpu_bf16.py > $OUT/r05_tn16_pytest.log 2>&1 || exit $?
tail -1 $OUT/r05_tn16_pytest.log
for lib in libdmrecblr.so ab_tn32.so libdmrecblr.so ab_tn32.so; do
  echo "== $lib" >> $OUT/r05_tn16_shapes.txt
  RECBLR_BF16_GEMM=1 RECBLR_LIB=$L/$lib timeout -k 10 300 python -u tools/bf16_gemm_probe.py >> $OUT/r05_tn16_shapes.txt 2>&1 || exit $?
done
for r in 1 2; do
  for m in auto 1 0; do
    echo "== $m" >> $OUT/r05_tn16_c5.txt
    RECBLR_BF16_GEMM=$m timeout -k 10 300 python -u tools/c5_step.py 6 >> $OUT/r05_tn16_c5.txt 2>&1 || exit $?
  done
done
grep -E "==|TN" $OUT/r05_tn16_shapes.txt; grep -v amdgpu.ids $OUT/r05_tn16_c5.txt
