#!/bin/bash
# round 5: the f16 CE kernels with 256 / 512 (shipped) / 1024 / 2048 target
# workgroups (more vocab splits per row block), alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/r05_ce_probe.txt
for r in 1 2 3; do
  for v in 256 shipped 1024 2048; do
    b=tools/bin/ce_h_probe_$v; [ $v = shipped ] && b=tools/bin/ce_h_probe
    echo -n "wgs=$v  " >> $OUT/r05_ce_probe.txt
    timeout -k 10 60 $b 2048 10544 128 30 >> $OUT/r05_ce_probe.txt 2>&1 || exit $?
  done
done
cat $OUT/r05_ce_probe.txt
