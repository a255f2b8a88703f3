#!/bin/bash
# round 5: static s_setprio 1 for the younger half of the 8-wave workgroups
# of the f16 NT / TN GEMMs (ab_prio.so; MI355X_MICROARCH.md, two waves per
# SIMD item 4) vs the shipped kernels: bench alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
SETTLE=8 bash tools/ab_gemm.sh 3 datamining_recblr_amd/lib/ab_prio.so datamining_recblr_amd/lib/libdmrecblr.so > $OUT/r05_prio_ab.txt 2>&1 || exit $?
cut -c1-60 $OUT/r05_prio_ab.txt
