mkdir -p gpurun_out
RECBLR_CE_GRADS=torch timeout -k 10 120 python tools/ce_bench.py 2048 10544 128 > gpurun_out/ce_f16.log 2>&1 &&
RECBLR_CE_GRADS=f16 timeout -k 10 120 python tools/ce_bench.py 2048 10544 128 >> gpurun_out/ce_f16.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_items.py tests/test_gpu_e2e.py >> gpurun_out/ce_f16.log 2>&1
