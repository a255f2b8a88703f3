# The CE backward products' cache-state probe, then the fused-GRL e2e tests
mkdir -p gpurun_out
timeout -k 10 180 tools/bin/ce_tn_probe 7 > gpurun_out/r04_ce_tn_probe.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_e2e.py -k fused_grl > gpurun_out/r04_pytest_fused_e2e.log 2>&1 || exit $?
