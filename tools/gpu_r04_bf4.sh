# NT bf16 kernel with tile-end stores and double-buffered fragments: tests,
# per-shape timings, configs[4] step A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04_bf4}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_gemm_bf16.py > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bf16_gemm_probe.py > gpurun_out/${T}_shapes.txt 2>&1 || exit $?
RECBLR_BF16_GEMM=1 timeout -k 10 300 python -u tools/c5_step.py 4 > gpurun_out/${T}_c5_on.txt 2>&1 || exit $?
RECBLR_BF16_GEMM=0 timeout -k 10 300 python -u tools/c5_step.py 4 > gpurun_out/${T}_c5_off.txt 2>&1
