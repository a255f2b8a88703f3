# The native Adam step: its GPU tests, then the bench step with it (optimizer
# time from the breakdown pass) against torch's fused Adam
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_optim.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/r03_adam_tests.log 2>&1 || exit $?
RECBLR_ADAM=native timeout -k 10 300 python bench.py --no-c5 --no-full-tail --no-cpu-baseline --no-ddp-ab \
    --settle-seconds 5 > gpurun_out/r03_adam_bench_native.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-c5 --no-full-tail --no-cpu-baseline --no-ddp-ab \
    --settle-seconds 5 > gpurun_out/r03_adam_bench_torch.log 2>&1
