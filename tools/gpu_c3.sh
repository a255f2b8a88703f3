mkdir -p gpurun_out
timeout -k 10 400 python bench.py --seq-len 50 --no-c5 --no-cpu-baseline --no-ddp-ab --settle-seconds 5 > gpurun_out/r03_c3_bench.log 2>&1
