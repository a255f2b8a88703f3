# NT GEMM tail: 256x64-tile round (default) vs the few-rows kernel
# (-DHN_TAIL_SMALL) vs the partial round in the persistent kernel
# (-DHN_NO_TAIL_SPLIT), alternated, at the bench's packed rows and at 3 whole rounds
mkdir -p gpurun_out
for r in 1 2; do
  for v in gemmbench_h gemmbench_h_tailsmall gemmbench_h_notail; do
    for m in 204632 196608; do
      echo "== $v M=$m round $r" >> gpurun_out/gemm_tail.log
      timeout -k 10 60 tools/bin/$v $m >> gpurun_out/gemm_tail.log 2>&1 || exit 1
    done
  done
done
