#!/bin/bash
# round 5: the ~30 us idle before the first gate-scan backward of each step:
# the timed loop's step sequence with and without bench.py's HIP events
# around the dominant kernel (--no-kernel-timing)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
for kt in on off; do
  X=""; [ $kt = off ] && X="--no-kernel-timing"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_w -o run \
    -- python3 bench.py --steps 10 --warmup 2 --settle-seconds 0 --no-cpu-baseline --no-full-tail \
    --no-c5 --no-ddp-ab $X > $OUT/prof_w_$kt.log 2>&1 || exit $?
  python tools/step_sequence.py $OUT/prof_w/run_kernel_trace.csv 8 3 > $OUT/r05_seq_timing_$kt.txt 2>&1
  rm -rf $OUT/prof_w
  head -2 $OUT/r05_seq_timing_$kt.txt; grep -E "k_gate_scan_bwd|k_pack_plan" $OUT/r05_seq_timing_$kt.txt | cut -c1-80
done
