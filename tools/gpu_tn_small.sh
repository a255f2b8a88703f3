# weight-gradient kernel at the gathered tail's rows: row-chunk count S
mkdir -p gpurun_out
for S in 8 16 32 64; do
  for m in 2048 6528; do
    echo "== S=$S M=$m" >> gpurun_out/tn_small.log
    GB_TN_S=$S timeout -k 10 60 tools/bin/gemmbench_h $m 2>&1 | grep -E "dW|tn total|WRONG" >> gpurun_out/tn_small.log || exit 1
  done
done
