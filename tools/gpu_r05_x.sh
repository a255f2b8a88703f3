#!/bin/bash
# round 5: keep the raw kernel trace of the bench's timed loop (compressed)
# to look at every dispatch around the idle before the first gate backward
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/prof_x -o run \
  -- python3 bench.py --steps 6 --warmup 2 --settle-seconds 0 --no-cpu-baseline --no-full-tail \
  --no-c5 --no-ddp-ab --no-kernel-timing > $OUT/prof_x.log 2>&1 || exit $?
ls $OUT/prof_x
gzip -c $OUT/prof_x/run_kernel_trace.csv > $OUT/r05_x_kernel_trace.csv.gz
[ -f $OUT/prof_x/run_memory_copy_trace.csv ] && gzip -c $OUT/prof_x/run_memory_copy_trace.csv > $OUT/r05_x_memcpy_trace.csv.gz
rm -rf $OUT/prof_x
ls -la $OUT/r05_x_*
