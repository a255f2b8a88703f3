mkdir -p gpurun_out
timeout -k 10 120 python tools/ce_grads_probe.py > gpurun_out/ce_probe.log 2>&1
