#!/bin/bash
# round 5: conv-forward tile loop + embedding plan + weight-image split:
# targeted tests, A/B against the previous conv forward, kernel trace, PMC
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
L=datamining_recblr_amd/lib
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_parity.py \
  tests/test_gpu_gemm_half.py tests/test_gpu_gemm.py -m gpu -q \
  -k "conv or embedding or weight_image or split or orientation" \
  --timeout 120 --timeout-method thread > $OUT/r05_b_pytest.log 2>&1 || exit $?
tail -2 $OUT/r05_b_pytest.log
timeout -k 10 900 bash tools/ab_multi.sh 2 $L/libdmrecblr.so $L/ab_convold.so \
  > $OUT/r05_b_ab.txt 2>&1 || exit $?
cat $OUT/r05_b_ab.txt
ARGS="--steps 10 --warmup 2 --settle-seconds 0 --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_b -o run \
  -- python3 bench.py $ARGS > $OUT/r05_b_prof.log 2>&1 || exit $?
cp $OUT/prof_b/run_kernel_stats.csv $OUT/r05_b_kernel_stats.csv
python tools/step_sequence.py $OUT/prof_b/run_kernel_trace.csv > $OUT/r05_b_step_sequence.txt 2>&1
rm -rf $OUT/prof_b
ARGS="--steps 3 --warmup 1 --settle-seconds 0 --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run \
  -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run \
  -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1 || exit $?
python tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write > $OUT/r05_b_pmc_traffic.json
rm -rf $OUT/pmc_fetch $OUT/pmc_write
