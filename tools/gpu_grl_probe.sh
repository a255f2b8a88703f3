mkdir -p gpurun_out
timeout -k 10 60 tools/bin/grlbench_p0 >> gpurun_out/grl_probe.txt 2>&1
