mkdir -p gpurun_out
timeout -k 10 60 tools/bin/gemmbench_h 2048 > gpurun_out/r03_v9_gemm2048.log 2>&1 &&
timeout -k 10 60 tools/bin/gemmbench_h 52000 > gpurun_out/r03_v9_gemm52000.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_gemm_half.py tests/test_gpu_gemm.py tests/test_gpu_e2e.py > gpurun_out/r03_v9_pytest.log 2>&1 &&
timeout -k 10 420 python bench.py --no-c5 --no-cpu-baseline > gpurun_out/r03_v9_bench.log 2>&1
