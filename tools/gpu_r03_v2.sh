mkdir -p gpurun_out
timeout -k 10 120 tools/bin/gemmbench_h 204632 > gpurun_out/r03_v2_gemmbench.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm_half.py > gpurun_out/r03_v2_pytest_gemm.log 2>&1 &&
timeout -k 10 360 python bench.py --no-c5 > gpurun_out/r03_v2_bench.log 2>&1 &&
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03_v2_pytest.log 2>&1
