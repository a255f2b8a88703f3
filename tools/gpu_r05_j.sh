#!/bin/bash
# round 5: where the ~80 us idle before the first gate-scan backward comes
# from: kernel + HIP API trace of the bench's timed loop (no counters)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
ARGS="--steps 10 --warmup 2 --settle-seconds 0 --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab --no-kernel-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/prof_j -o run \
  -- python3 bench.py $ARGS > $OUT/r05_j_prof.log 2>&1 || exit $?
python tools/step_sequence.py $OUT/prof_j/run_kernel_trace.csv 8 3 > $OUT/r05_j_step_sequence.txt 2>&1
python tools/host_gap.py $OUT/prof_j/run 6 30 > $OUT/r05_j_host_gap.txt 2>&1 && python tools/host_gap.py $OUT/prof_j/run 9 30 > $OUT/r05_j_host_gap9.txt 2>&1
rm -rf $OUT/prof_j
head -2 $OUT/r05_j_step_sequence.txt; cat $OUT/r05_j_host_gap.txt | head -60
