#!/bin/bash
# ab_multi.sh ROUNDS LIB... — alternate bench.py runs over several builds (RECBLR_LIB)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq 1 $rounds); do
  for lib in "$@"; do
    RECBLR_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-c5 --no-full-tail --settle-seconds ${SETTLE:-8} > gpurun_out/ab.log 2>&1 || exit 1
    tail -1 gpurun_out/ab.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('$(basename $lib)', d['value'], d['ms_per_step'], 'path', k['scan_conv_gate_path']['frac'], ' '.join('%s=%.3f'%(n[3:],v['frac']) for n,v in k.items() if n.startswith('rb_conv') or n.startswith('rb_gate')))"
  done
done
