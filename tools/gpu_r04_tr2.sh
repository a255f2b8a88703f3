# The even-swizzle transposed gather: the gather probe over both swizzles,
# then the item tests and the whole-step e2e tests (all, no -x)
mkdir -p gpurun_out
timeout -k 10 60 tools/bin/tr16_gather_probe > gpurun_out/r04_tr16_gather_probe.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
    tests/test_gpu_items.py > gpurun_out/r04_ce_pytest_items_ev.log 2>&1 || exit $?
RECBLR_CE_GRADS=fused timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_e2e.py > gpurun_out/r04_ce_pytest_e2e_ev.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab \
    > gpurun_out/r04_ce_bench_ev.log 2>&1
