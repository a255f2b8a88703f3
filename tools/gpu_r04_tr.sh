# ds_read_b64_tr_b16 semantics probe, then the item tests (all, no -x)
mkdir -p gpurun_out
timeout -k 10 60 tools/bin/tr16_probe > gpurun_out/r04_tr16_probe.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
    tests/test_gpu_items.py > gpurun_out/r04_ce_pytest_items2.log 2>&1
exit 0
