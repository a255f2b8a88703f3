# The gates GEMM with the BD-LRU epilogue: its own tests, the e2e parity with
# it engaged, then the default bench line and the two-launch A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04_gate
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_gate_gemm.py tests/test_gpu_blocks.py::test_pack_plan_matches_torch \
    > gpurun_out/${T}_pytest_gate.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_e2e.py > gpurun_out/${T}_pytest_e2e.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab \
    > gpurun_out/${T}_bench_on.log 2>&1 || exit $?
RECBLR_GATE_GEMM=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-tail --no-c5 \
    --no-ddp-ab > gpurun_out/${T}_bench_off.log 2>&1 || exit $?
