# bf16 projection kernels, second form (NT: A two k-steps ahead through 3
# stages; TN: 32-row k-steps, 4 stages): tests, configs[4] A/B, kernel
# summary; the transposed-read row dump
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04_bf2
timeout -k 10 60 tools/bin/tr16_gather_probe > gpurun_out/r04_tr16_gather_probe2.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_gemm_bf16.py > gpurun_out/${T}_pytest.log 2>&1 || exit $?
RECBLR_BF16_GEMM=1 timeout -k 10 300 python -u tools/c5_step.py 4 > gpurun_out/${T}_c5_on.txt 2>&1 || exit $?
RECBLR_BF16_GEMM=0 timeout -k 10 300 python -u tools/c5_step.py 4 > gpurun_out/${T}_c5_off.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bf -o c5 \
    -- python3 tools/c5_step.py 3 > gpurun_out/${T}_prof.log 2>&1 || exit $?
cp gpurun_out/prof_bf/c5_kernel_stats.csv gpurun_out/${T}_c5_kernel_stats.csv
rm -rf gpurun_out/prof_bf
