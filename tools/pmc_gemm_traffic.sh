#!/bin/bash
# HBM traffic per NT GEMM shape: FETCH_SIZE and WRITE_SIZE passes (one each,
# as gfx950 requires) over tools/bin/gemmbench_h_<variant>; per-dispatch CSVs
# summarised by tools/pmc_gemm_traffic.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
for v in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $OUT/pmcg_${v}_$c -o run \
      -- tools/bin/gemmbench_h_$v > $OUT/pmcg_${v}_$c.log 2>&1 || exit $?
  done
done
