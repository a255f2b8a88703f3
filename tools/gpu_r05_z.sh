#!/bin/bash
# round 5: kernel summary of the configs[4] step (per-shape bf16 default,
# TunableOp table) — where its 21.3 ms go
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_z -o c5 \
  -- python3 tools/c5_step.py 4 > $OUT/r05_z_c5.log 2>&1 || exit $?
cp $OUT/prof_z/c5_kernel_stats.csv $OUT/${T:-r05}_c5_kernel_stats.csv
rm -rf $OUT/prof_z
tail -2 $OUT/r05_z_c5.log
