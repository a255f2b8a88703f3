# Counting-sort embedding plan in three launches, last-layer y in batch order
# (no gather / index_add pair): block + e2e tests, bench line, step sequence
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04_v4
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_e2e.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_train.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-c5 --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
    -- python3 bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab > gpurun_out/${T}_prof.log 2>&1
rc=$?
cp gpurun_out/prof/bench_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv 2>/dev/null
python tools/step_sequence.py gpurun_out/prof/bench_kernel_trace.csv 10 > gpurun_out/${T}_step_sequence.txt 2>&1
rm -rf gpurun_out/prof
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/bin/mix_bench 204632 7 > gpurun_out/${T}_mix_bench.txt 2>&1
