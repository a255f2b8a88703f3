# embedding backward on rocPRIM Onesweep: its tests, then the bench step's
# kernel summary (the sort kernels' share)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_blocks.py tests/test_gpu_e2e.py > gpurun_out/emb_tests.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
    -- python3 bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab > gpurun_out/emb_bench.txt 2>&1
rc=$?
cp gpurun_out/prof/bench_kernel_stats.csv gpurun_out/emb_kernel_stats.csv 2>/dev/null
rm -rf gpurun_out/prof
exit $rc
