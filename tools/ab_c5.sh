#!/bin/bash
# ab_c5.sh LIB_A LIB_B — the configs[4] (long_seq_bf16) run of bench.py under two builds
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for lib in "$1" "$2"; do
  RECBLR_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-tail --steps 5 --warmup 2 --settle-seconds 3 > gpurun_out/abc5.log 2>&1 || exit 1
  tail -1 gpurun_out/abc5.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())['long_seq_bf16']
print('$(basename $lib)', d['value'], d['ms_per_step'], 'path', d['scan_conv_gate_path']['frac'], ' '.join('%s=%.3f'%(n[3:],v['frac']) for n,v in d['scan_conv_gate_path']['kernels'].items()))"
done
