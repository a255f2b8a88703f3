#!/bin/bash
# round 5: bf16 NT on v_mfma_f32_16x16x32_bf16 (product build) against the
# 32x32x16 kernel (ab_bfold.so): tests, per-shape timings, configs[4] step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
L=datamining_recblr_amd/lib
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_gemm_bf16.py tests/test_gpu_bf16.py > $OUT/r05_mf16_pytest.log 2>&1 || exit $?
tail -2 $OUT/r05_mf16_pytest.log
for lib in libdmrecblr.so ab_bfold.so libdmrecblr.so ab_bfold.so; do
  echo "== $lib" >> $OUT/r05_mf16_shapes.txt
  RECBLR_LIB=$L/$lib timeout -k 10 300 python -u tools/bf16_gemm_probe.py >> $OUT/r05_mf16_shapes.txt 2>&1 || exit $?
done
for lib in libdmrecblr.so ab_bfold.so libdmrecblr.so; do
  echo "== $lib" >> $OUT/r05_mf16_c5.txt
  RECBLR_LIB=$L/$lib RECBLR_BF16_GEMM=1 timeout -k 10 300 python -u tools/c5_step.py 4 >> $OUT/r05_mf16_c5.txt 2>&1 || exit $?
done
echo "== hipBLASLt" >> $OUT/r05_mf16_c5.txt
RECBLR_BF16_GEMM=0 timeout -k 10 300 python -u tools/c5_step.py 4 >> $OUT/r05_mf16_c5.txt 2>&1
grep -v amdgpu.ids $OUT/r05_mf16_shapes.txt; grep -v amdgpu.ids $OUT/r05_mf16_c5.txt
