# weight-gradient kernel: role-split (producer/consumer) variant vs the current one, alternated
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in gemmbench_h gemmbench_h_tn16; do
    echo "== $v round $r" >> gpurun_out/tn_pc.log
    timeout -k 10 60 tools/bin/$v 204632 2>&1 | grep -E "dW|tn total|WRONG" >> gpurun_out/tn_pc.log || exit 1
  done
done
