#!/bin/bash
# round 5: the f16 split's share of the NT GEMM (timing-only ablation build,
# tools/bin/gemm_ab_nosplit), the unrolled chunked column sum (tests + trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_parity.py tests/test_gpu_e2e.py \
  -m gpu -q -k "colsum or conv or gate or train_step or pad" \
  --timeout 120 --timeout-method thread > $OUT/r05_c_pytest.log 2>&1 || exit $?
tail -2 $OUT/r05_c_pytest.log
for v in cur nosplit cur nosplit; do
  echo "== $v" >> $OUT/r05_nosplit_ab.txt
  timeout -k 10 120 tools/bin/gemm_ab_$v 204632 9 >> $OUT/r05_nosplit_ab.txt 2>&1 || exit $?
done
grep -E "==|total" $OUT/r05_nosplit_ab.txt
ARGS="--steps 10 --warmup 2 --settle-seconds 0 --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c -o run \
  -- python3 bench.py $ARGS > $OUT/r05_c_prof.log 2>&1 || exit $?
cp $OUT/prof_c/run_kernel_stats.csv $OUT/r05_c_kernel_stats.csv
python tools/step_sequence.py $OUT/prof_c/run_kernel_trace.csv > $OUT/r05_c_step_sequence.txt 2>&1
rm -rf $OUT/prof_c
head -2 $OUT/r05_c_step_sequence.txt
