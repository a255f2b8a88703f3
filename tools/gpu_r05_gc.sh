#!/bin/bash
# round 5: the bf16 gate backward in two channel passes — its GPU tests, then
# the configs[4] step alternated against the previous build (ab_gsold.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_parity.py tests/test_gpu_gemm_bf16.py -x -q --timeout 200 --timeout-method thread > $OUT/r05_gc_pytest.log 2>&1 || exit $?
tail -1 $OUT/r05_gc_pytest.log
: > $OUT/r05_gc_c5.txt
for r in 1 2 3; do
  for lib in datamining_recblr_amd/lib/libdmrecblr.so datamining_recblr_amd/lib/ab_gsold.so; do
    echo "== $(basename $lib)" >> $OUT/r05_gc_c5.txt
    RECBLR_LIB=$lib timeout -k 10 200 python tools/c5_step.py 4 >> $OUT/r05_gc_c5.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $OUT/r05_gc_c5.txt
