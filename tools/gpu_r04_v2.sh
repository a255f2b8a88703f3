# TN per-column redo: its tests and the GEMM suites, then the bench line with
# the backward-order A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_half.py tests/test_gpu_gemm.py tests/test_gpu_items.py tests/test_gpu_e2e.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/r04_v2_pytest_gemm.log 2>&1 || exit $?
timeout -k 10 700 python bench.py --no-c5 --no-cpu-baseline > gpurun_out/r04_v2_bench.log 2>&1
