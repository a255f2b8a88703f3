#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench and a rocprofv3
# kernel-trace of the bench.  Stops at the first fault/abort/timeout
# (exit status other than 0 = pass or 1 = test failures).
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }

timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
ok $rc || exit $rc
[ -n "$TESTS_ONLY" ] && exit $rc

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log
ok $rc || exit $rc

timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.log
ok $rc || exit $rc

if [ -z "$NO_PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench \
      -- python3 bench.py --steps 5 --warmup 2 --settle-seconds 4 --no-cpu-baseline --no-full-tail --no-c5 > $OUT/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 $OUT/prof.log
fi
exit $rc
