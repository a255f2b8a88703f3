#!/bin/bash
# round 5: the packed layout's host -> device copy on a copy stream ahead of
# the step (RECBLR_COPY_AHEAD=1, new default) vs on the current stream (=0):
# the multi-step GPU tests, a kernel-trace look at the step start, then the
# bench alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_optim.py tests/test_gpu_timed_step.py tests/test_gpu_e2e.py tests/test_gpu_ddp.py tests/test_gpu_eval.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > $OUT/r05_ca_pytest.log 2>&1 || exit $?
tail -1 $OUT/r05_ca_pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/prof_ca -o run \
  -- python3 bench.py --steps 10 --warmup 2 --settle-seconds 0 --no-cpu-baseline --no-full-tail \
  --no-c5 --no-ddp-ab --no-kernel-timing > $OUT/r05_ca_prof.log 2>&1 || exit $?
python tools/step_sequence.py $OUT/prof_ca/run_kernel_trace.csv 8 3 > $OUT/r05_ca_step_sequence.txt 2>&1
rm -rf $OUT/prof_ca
head -6 $OUT/r05_ca_step_sequence.txt
SETTLE=8 bash tools/ab_env.sh "RECBLR_COPY_AHEAD=1" "RECBLR_COPY_AHEAD=0" 3 > $OUT/r05_ca_ab.txt 2>&1 || exit $?
cut -c1-60 $OUT/r05_ca_ab.txt
