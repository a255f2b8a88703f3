mkdir -p gpurun_out
for p in 0 1 2 4 8 15; do
  timeout -k 10 60 tools/bin/grlbench_p$p >> gpurun_out/grl_probe.txt 2>&1 || exit 1
done
GRL_FIXED=1 timeout -k 10 60 tools/bin/grlbench_p0 >> gpurun_out/grl_probe.txt 2>&1
