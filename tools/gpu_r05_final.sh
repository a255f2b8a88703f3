#!/bin/bash
# Round-5 closing evidence: the whole GPU suite, smoke, the default bench
# line, the rocprof kernel summary + the timed loop's step sequence, and the
# PMC passes (HBM traffic, MFMA busy, clocks) whose summaries the bench line
# cites.  T=<tag> names the outputs (default r05_final); PART=1 runs only the
# suite and smoke, PART=2 only the rest (two calls under gpurun's limit).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
T=${T:-r05_final}
PART=${PART:-all}
if [ "$PART" != 2 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > $OUT/${T}_pytest_gpu.log 2>&1 || exit $?
tail -1 $OUT/${T}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${T}_smoke.log 2>&1 || exit $?
tail -2 $OUT/${T}_smoke.log
fi
[ "$PART" = 1 ] && exit 0
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench \
    -- python3 bench.py --steps 10 --warmup 2 --settle-seconds 0 --no-cpu-baseline --no-full-tail \
    --no-c5 --no-ddp-ab > $OUT/${T}_prof.log 2>&1 || exit $?
cp $OUT/prof/bench_kernel_stats.csv $OUT/${T}_kernel_stats.csv
python tools/step_sequence.py $OUT/prof/bench_kernel_trace.csv 8 3 > $OUT/${T}_step_sequence.txt 2>&1
rm -rf $OUT/prof
bash tools/pmc_all.sh || exit $?
cp $OUT/pmc_traffic.json $OUT/${T}_pmc_traffic.json
cp $OUT/pmc_mfma.json $OUT/${T}_pmc_mfma.json
rm -rf $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_mfma
# the bench line cites the newest profiles/*_pmc_*.json: this lease's
cp $OUT/${T}_pmc_traffic.json profiles/${T}_pmc_traffic.json
cp $OUT/${T}_pmc_mfma.json profiles/${T}_pmc_mfma.json
timeout -k 10 900 python bench.py > $OUT/${T}_bench.log 2>&1 || exit $?
tail -c 400 $OUT/${T}_bench.log
