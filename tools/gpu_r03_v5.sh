mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py > gpurun_out/r03_v5_fused.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_e2e.py tests/test_gpu_eval.py tests/test_gpu_ddp.py > gpurun_out/r03_v5_e2e.log 2>&1 &&
timeout -k 10 420 python bench.py --no-c5 --no-cpu-baseline > gpurun_out/r03_v5_bench.log 2>&1
