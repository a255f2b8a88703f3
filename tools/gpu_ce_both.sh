# CE backward on both layouts of P: tests, bench, rocprof (RECBLR_TN_FEW=1: no library GEMM)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_items.py tests/test_gpu_e2e.py tests/test_gpu_gemm_half.py > gpurun_out/ceb_tests.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline --no-full-tail --no-c5 > gpurun_out/ceb_bench.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline --no-full-tail --no-c5 > gpurun_out/ceb_bench_tnfew.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
    -- python3 bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab > gpurun_out/ceb_prof.txt 2>&1
rc=$?
cp gpurun_out/prof/bench_kernel_stats.csv gpurun_out/ceb_kernel_stats.csv 2>/dev/null
rm -rf gpurun_out/prof
exit $rc
