#!/bin/bash
# ab_gemm.sh ROUNDS LIB... — alternate bench.py runs over builds (RECBLR_LIB)
# and print the step, the projection GEMMs' time per step and each shape's
# kernel time from the bench's gemm.pattern leg
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq 1 $rounds); do
  for lib in "$@"; do
    RECBLR_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-c5 --no-full-tail --no-ddp-ab --settle-seconds ${SETTLE:-8} > gpurun_out/ab.log 2>&1 || exit 1
    tail -1 gpurun_out/ab.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); g=d['gemm']; p=g.get('pattern') or {}
print('$(basename $lib)', d['ms_per_step'], 'gemm_ms', g['ms_per_step'], ' '.join('%s=%.1f'%(n,v['kernel_us']) for n,v in p.get('shapes',{}).items()))"
  done
done
