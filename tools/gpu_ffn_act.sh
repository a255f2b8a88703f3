# FeedForward activation in w_1's GEMM epilogue: parity tests, the GEMM
# tests, the e2e oracle tests, then the bench line with the on-lease A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_half.py tests/test_gpu_blocks.py tests/test_gpu_e2e.py \
    -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r03_ffnact_tests.log 2>&1 || exit $?
timeout -k 10 700 python bench.py --no-c5 > gpurun_out/r03_ffnact_bench.log 2>&1
