# Round-4 start: the GPU suite on the current tree, smoke, the default bench
# line (with the Adam A/B), and the rocprof kernel summary of the bench step
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/r04_v0_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_v0_smoke.log 2>&1 || exit $?
timeout -k 10 700 python bench.py > gpurun_out/r04_v0_bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
    -- python3 bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab > gpurun_out/r04_v0_prof.log 2>&1
rc=$?
cp gpurun_out/prof/bench_kernel_stats.csv gpurun_out/r04_v0_kernel_stats.csv 2>/dev/null
python tools/step_sequence.py gpurun_out/prof/bench_kernel_trace.csv 10 > gpurun_out/r04_v0_step_sequence.txt 2>&1
rm -rf gpurun_out/prof
exit $rc
