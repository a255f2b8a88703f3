# The P-free CE backward (rb_item_ce_bwd_h): item tests, e2e parity, the
# bench with it (default) and with RECBLR_CE_GRADS=f16, the old path's probe
mkdir -p gpurun_out
T=r04_ce
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_items.py > gpurun_out/${T}_pytest_items.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_e2e.py > gpurun_out/${T}_pytest_e2e.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab \
    > gpurun_out/${T}_bench_fused.log 2>&1 || exit $?
RECBLR_CE_GRADS=f16 timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-tail --no-c5 \
    --no-ddp-ab > gpurun_out/${T}_bench_f16.log 2>&1 || exit $?
RECBLR_CE_GRADS=f16 timeout -k 10 300 python -u tools/ce_step_probe.py \
    > gpurun_out/r04_ce_step_probe.txt 2>&1 || exit $?
