# gathered-tail GEMMs (B = 2048 rows): few-rows kernel vs 256x64 tiles of the persistent kernel
mkdir -p gpurun_out
for r in 1 2; do
  for v in gemmbench_h gemmbench_h_smallnb2; do
    for m in 2048 8192; do
      echo "== $v M=$m round $r" >> gpurun_out/gemm_small.log
      timeout -k 10 60 tools/bin/$v $m >> gpurun_out/gemm_small.log 2>&1 || exit 1
    done
  done
done
