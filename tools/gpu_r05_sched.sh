#!/bin/bash
# round 5: the whole library built with LLVM's alternative AMDGPU machine
# schedulers (-mllvm -amdgpu-sched-strategy=max-ilp / max-memory-clause) vs
# the default: bench alternated (step and per-shape GEMM times)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
SETTLE=8 bash tools/ab_gemm.sh 2 datamining_recblr_amd/lib/ab_max-ilp.so datamining_recblr_amd/lib/ab_max-memory-clause.so datamining_recblr_amd/lib/libdmrecblr.so > $OUT/r05_sched_ab.txt 2>&1 || exit $?
cut -c1-64 $OUT/r05_sched_ab.txt
