mkdir -p gpurun_out
timeout -k 10 120 python tools/ce_bench.py 2048 10544 128 > gpurun_out/r03_v6_ce.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ddp.py > gpurun_out/r03_v6_ddp.log 2>&1 &&
timeout -k 10 420 python bench.py --no-c5 --no-cpu-baseline > gpurun_out/r03_v6_bench.log 2>&1
