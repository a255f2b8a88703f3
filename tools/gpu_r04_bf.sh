# bf16 projection kernels (configs[4]) + the even-swizzle CE gather:
# probe, tests, configs[4] step A/B and its kernel summary.  A failing test
# (pytest rc 1) does not stop the script; anything worse does.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04_bf
ok() { local rc=$1; [ "$rc" -le 1 ] || exit "$rc"; }
timeout -k 10 60 tools/bin/tr16_gather_probe > gpurun_out/r04_tr16_gather_probe.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread \
    tests/test_gpu_gemm_bf16.py tests/test_gpu_bf16.py > gpurun_out/${T}_pytest.log 2>&1; ok $?
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
    tests/test_gpu_items.py > gpurun_out/${T}_pytest_items_ev.log 2>&1; ok $?
RECBLR_BF16_GEMM=1 timeout -k 10 300 python -u tools/c5_step.py 4 > gpurun_out/${T}_c5_on.txt 2>&1 || exit $?
RECBLR_BF16_GEMM=0 timeout -k 10 300 python -u tools/c5_step.py 4 > gpurun_out/${T}_c5_off.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bf -o c5 \
    -- python3 tools/c5_step.py 3 > gpurun_out/${T}_prof.log 2>&1 || exit $?
cp gpurun_out/prof_bf/c5_kernel_stats.csv gpurun_out/${T}_c5_kernel_stats.csv
rm -rf gpurun_out/prof_bf
