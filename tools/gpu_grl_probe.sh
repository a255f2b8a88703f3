# grlbench: the fused GRL kernels and their ablation builds (-DGRL_PROBE),
# then the SQ counters (tools/pmc_grl.sh)
mkdir -p gpurun_out
for p in 0 1 2 4 8 16 32 40; do
  timeout -k 10 60 tools/bin/grlbench_p$p >> gpurun_out/grl_probe.txt 2>&1 || exit 1
done
bash tools/pmc_grl.sh
