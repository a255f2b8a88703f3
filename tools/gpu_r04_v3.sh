# Counting-sort embedding plan: the block tests (incl. counting vs radix
# plan), the e2e suite, then the bench line and the step sequence
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_e2e.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/r04_v3_pytest.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
    -- python3 bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab > gpurun_out/r04_v3_prof.log 2>&1
rc=$?
cp gpurun_out/prof/bench_kernel_stats.csv gpurun_out/r04_v3_kernel_stats.csv 2>/dev/null
python tools/step_sequence.py gpurun_out/prof/bench_kernel_trace.csv 10 > gpurun_out/r04_v3_step_sequence.txt 2>&1
rm -rf gpurun_out/prof
exit $rc
