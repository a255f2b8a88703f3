#!/bin/bash
# ab_env.sh "ENV_A" "ENV_B" [ROUNDS] — alternate bench.py runs under two
# environment settings (e.g. RECBLR_CONV_ROWS=0 vs 1), same library
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in $(seq 1 ${3:-2}); do
  for e in "$1" "$2"; do
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-c5 --no-full-tail --settle-seconds ${SETTLE:-10} > gpurun_out/ab.log 2>&1 || exit 1
    tail -1 gpurun_out/ab.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('$e', d['value'], d['ms_per_step'], 'path', k['scan_conv_gate_path']['frac'], ' '.join('%s=%.3f'%(n[3:],v['frac']) for n,v in k.items() if n.startswith('rb_')))"
  done
done
