mkdir -p gpurun_out
timeout -k 10 120 tools/bin/gemmbench_h 204632 > gpurun_out/r03_gemmbench_tail.log 2>&1 &&
timeout -k 10 120 tools/bin/gemmbench_h 196608 >> gpurun_out/r03_gemmbench_tail.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm_half.py > gpurun_out/r03_v1_pytest_gemm.log 2>&1 &&
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03_v1_pytest.log 2>&1 &&
timeout -k 10 360 python bench.py > gpurun_out/r03_v1_bench.log 2>&1
