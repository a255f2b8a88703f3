#!/bin/bash
# round 5: bf16 NT with the barrier between the k32 halves (A 3 steps ahead;
# product build, early half-0 reads) against the previous commit (ab_bfc1)
# and the late-read/bias-before-DMA variant (ab_bfl1): tests, shapes, step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
L=datamining_recblr_amd/lib
mkdir -p $OUT
for lib in libdmrecblr.so ab_bfl1.so; do
  RECBLR_LIB=$L/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      tests/test_gpu_gemm_bf16.py tests/test_gpu_bf16.py > $OUT/r05_bfmid_pytest_$lib.log 2>&1 || exit $?
  tail -1 $OUT/r05_bfmid_pytest_$lib.log
done
for lib in libdmrecblr.so ab_bfc1.so ab_bfl1.so libdmrecblr.so ab_bfc1.so ab_bfl1.so; do
  echo "== $lib" >> $OUT/r05_bfmid_shapes.txt
  RECBLR_LIB=$L/$lib timeout -k 10 300 python -u tools/bf16_gemm_probe.py >> $OUT/r05_bfmid_shapes.txt 2>&1 || exit $?
done
for lib in libdmrecblr.so ab_bfc1.so ab_bfl1.so libdmrecblr.so ab_bfc1.so; do
  echo "== $lib" >> $OUT/r05_bfmid_c5.txt
  RECBLR_LIB=$L/$lib RECBLR_BF16_GEMM=1 timeout -k 10 300 python -u tools/c5_step.py 4 >> $OUT/r05_bfmid_c5.txt 2>&1 || exit $?
done
echo "== hipBLASLt" >> $OUT/r05_bfmid_c5.txt
RECBLR_BF16_GEMM=0 timeout -k 10 300 python -u tools/c5_step.py 4 >> $OUT/r05_bfmid_c5.txt 2>&1
grep -v amdgpu.ids $OUT/r05_bfmid_c5.txt
