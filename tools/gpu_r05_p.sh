#!/bin/bash
# round 5: configs[4] with the weight gradients back on the library in the
# per-shape mode: tests, C5 step per mode alternated, the bench's c5 object
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_gemm_bf16.py tests/test_gpu_bf16.py > $OUT/r05_bfauto2_pytest.log 2>&1 || exit $?
tail -1 $OUT/r05_bfauto2_pytest.log
for r in 1 2 3; do
  for m in auto 1 0; do
    echo "== $m" >> $OUT/r05_bfauto2_c5.txt
    RECBLR_BF16_GEMM=$m timeout -k 10 300 python -u tools/c5_step.py 6 >> $OUT/r05_bfauto2_c5.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $OUT/r05_bfauto2_c5.txt
timeout -k 10 600 python bench.py --no-cpu-baseline --no-full-tail --no-ddp-ab > $OUT/r05_bfauto2_bench.log 2>&1 || exit $?
tail -1 $OUT/r05_bfauto2_bench.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['long_seq_bf16']
print(d['value'], d['ms_per_step'], 'c5', c['ms_per_step'], json.dumps(c['projection_gemms_ab']))"
