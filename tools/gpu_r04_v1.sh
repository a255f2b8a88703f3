# Round-4 launch cuts: GEMM main + tail phases in one launch, one-launch
# chunked column sums, fused pad-prefix kernels, CE pad columns in-kernel,
# native Adam by default: the GPU suite, the bench line, the step sequence
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/r04_v1_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-c5 --no-cpu-baseline > gpurun_out/r04_v1_bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
    -- python3 bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab > gpurun_out/r04_v1_prof.log 2>&1
rc=$?
cp gpurun_out/prof/bench_kernel_stats.csv gpurun_out/r04_v1_kernel_stats.csv 2>/dev/null
python tools/step_sequence.py gpurun_out/prof/bench_kernel_trace.csv 10 > gpurun_out/r04_v1_step_sequence.txt 2>&1
rm -rf gpurun_out/prof
exit $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/bin/gemm_epi 204632 9 > gpurun_out/r04_gemm_epi.txt 2>&1
