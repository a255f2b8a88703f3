#!/bin/bash
# round 5: the CE forward with 3 item tiles in flight (product) against the
# double-buffered stream (ab_ceold): tests, kernel timing, bench A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
L=datamining_recblr_amd/lib
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_items.py > $OUT/r05_cedeep_pytest.log 2>&1 || exit $?
tail -1 $OUT/r05_cedeep_pytest.log
for lib in libdmrecblr.so ab_ceold.so libdmrecblr.so ab_ceold.so; do
  for shp in "2048 10544 128" "2048 10544 64" "2048 10544 256" "4096 50000 128"; do
    echo -n "$lib  " >> $OUT/r05_cedeep_probe.txt
    RECBLR_LIB=$L/$lib timeout -k 10 120 python -u tools/ce_fwd_probe.py $shp 2>&1 | grep ce_fwd >> $OUT/r05_cedeep_probe.txt || exit $?
  done
done
cat $OUT/r05_cedeep_probe.txt
SETTLE=5 timeout -k 10 900 bash tools/ab_gemm.sh 2 $L/libdmrecblr.so $L/ab_ceold.so > $OUT/r05_cedeep_bench_ab.txt 2>&1 || exit $?
cut -c1-60 $OUT/r05_cedeep_bench_ab.txt
