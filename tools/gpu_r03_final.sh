mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python bench.py > gpurun_out/r03_v10_bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
    -- python3 bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab > gpurun_out/r03_v10_prof.log 2>&1
rc=$?
cp gpurun_out/prof/bench_kernel_stats.csv gpurun_out/r03_v10_kernel_stats.csv 2>/dev/null
rm -rf gpurun_out/prof
exit $rc
