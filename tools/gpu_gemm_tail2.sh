mkdir -p gpurun_out
for r in 1 2; do
  for v in gemmbench_h gemmbench_h_tail2; do
    echo "== $v round $r" >> gpurun_out/gemm_tail2.log
    timeout -k 10 60 tools/bin/$v 204632 2>&1 | grep -vE "dW|tn total" >> gpurun_out/gemm_tail2.log || exit 1
  done
done
