#!/bin/bash
# round 5: conv-forward tile mapping A/B, HIP-graph probe, PMC traffic of the
# headline step (FETCH / WRITE passes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
L=datamining_recblr_amd/lib
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_parity.py -m gpu -q -k "conv or embedding" \
  --timeout 120 --timeout-method thread > $OUT/r05_a_pytest_conv.log 2>&1 || exit $?
tail -2 $OUT/r05_a_pytest_conv.log
timeout -k 10 900 bash tools/ab_multi.sh 2 $L/libdmrecblr.so $L/ab_convold.so $L/ab_convtc8.so \
  > $OUT/r05_conv_ab.txt 2>&1 || exit $?
cat $OUT/r05_conv_ab.txt
ARGS="--steps 3 --warmup 1 --settle-seconds 0 --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run \
  -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run \
  -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1 || exit $?
python tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write > $OUT/r05_pmc_traffic.json
rm -rf $OUT/pmc_fetch $OUT/pmc_write
timeout -k 10 300 python -u tools/graph_probe.py > $OUT/r05_graph_probe.txt 2>&1
rc=$?; tail -1 $OUT/r05_graph_probe.txt; exit $rc
