#!/bin/bash
# One GPU-box session: parity tests, smoke, the bf16 error probe, the bench
# and a rocprofv3 kernel-trace of the bench on the same lease.  Stops at the
# first fault/abort/timeout (exit status other than 0 = pass or 1 = test
# failures).  TESTS_ONLY=1: tests only; NO_PROF=1: skip rocprof;
# PYTEST_ARGS / BENCH_ARGS pass through.
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }

if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread \
      ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
  ok $rc || exit $rc
  [ -n "$TESTS_ONLY" ] && exit $rc

  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log
  ok $rc || exit $rc
fi

if [ -n "$BF16_ERR" ]; then
  timeout -k 10 300 python tools/bf16_err.py > $OUT/bf16_err.json 2> $OUT/bf16_err.log
  rc=$?; echo "bf16_err rc=$rc"; cat $OUT/bf16_err.json
  ok $rc || exit $rc
fi

timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 $OUT/bench.log
ok $rc || exit $rc

if [ -z "$NO_PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench \
      -- python3 bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab > $OUT/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -c 300 $OUT/prof.log
  # keep the summaries, drop the (large) per-dispatch trace
  cp $OUT/prof/bench_kernel_stats.csv $OUT/prof_kernel_stats.csv 2>/dev/null
  rm -rf $OUT/prof
fi
exit $rc
