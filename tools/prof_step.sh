#!/bin/bash
# prof_step.sh TAG — rocprofv3 kernel trace + stats of a short bench run
# (the timed loop's step sequence: tools/step_sequence.py), then the PMC
# passes of tools/pmc_all.sh; everything under gpurun_out/TAG_*.
set -o pipefail
TAG=${1:-prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
ARGS="--steps 10 --warmup 2 --settle-seconds 0 --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_kt -o run \
  -- python3 bench.py $ARGS > $OUT/${TAG}_prof.log 2>&1 || exit $?
KT=$(ls $OUT/${TAG}_kt/*/run_kernel_trace.csv $OUT/${TAG}_kt/run_kernel_trace.csv 2>/dev/null | head -1)
ST=$(ls $OUT/${TAG}_kt/*/run_kernel_stats.csv $OUT/${TAG}_kt/run_kernel_stats.csv 2>/dev/null | head -1)
cp "$ST" $OUT/${TAG}_kernel_stats.csv
python tools/step_sequence.py "$KT" 10 > $OUT/${TAG}_step_sequence.txt || exit $?
rm -rf $OUT/${TAG}_kt
if [ "${PMC:-1}" = 1 ]; then
  bash tools/pmc_all.sh && cp $OUT/pmc_traffic.json $OUT/${TAG}_pmc_traffic.json && \
    cp $OUT/pmc_mfma.json $OUT/${TAG}_pmc_mfma.json && rm -rf $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_mfma
fi
