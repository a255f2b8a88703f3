#!/bin/bash
# round 5: TunableOp search over the configs[4] projections that the
# per-shape mode leaves on the library (in / gates input gradients, the
# three weight gradients' batched GEMMs), merged into the shipped table,
# then the C5 step with and without the table, alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
cp datamining_recblr_amd/tuning/gemm_gfx950.csv $OUT/table_before.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=0 \
  PYTORCH_TUNABLEOP_FILENAME=$OUT/tune_c5.csv RECBLR_TUNED_GEMMS=0 \
  timeout -k 10 600 python -u tools/c5_step.py 2 > $OUT/r05_tune_c5.txt 2>&1 || exit $?
ls $OUT | grep tune_c5
python tools/tunable_merge.py $(ls $OUT/tune_c5*.csv | head -1) > $OUT/r05_tune_merge.txt 2>&1 || exit $?
cat $OUT/r05_tune_merge.txt
cp datamining_recblr_amd/tuning/gemm_gfx950.csv $OUT/table_after.csv
for r in 1 2 3; do
  for t in 1 0; do
    echo "== tuned=$t" >> $OUT/r05_tune_c5_ab.txt
    RECBLR_TUNED_GEMMS=$t timeout -k 10 300 python -u tools/c5_step.py 6 >> $OUT/r05_tune_c5_ab.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $OUT/r05_tune_c5_ab.txt
