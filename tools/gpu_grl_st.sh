mkdir -p gpurun_out
timeout -k 10 60 tools/bin/grlbench_p0 > gpurun_out/grl_st.txt 2>&1 &&
timeout -k 10 60 tools/bin/grlbench_st >> gpurun_out/grl_st.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py > gpurun_out/grl_fused_tests.log 2>&1
