# Weight-gradient GEMM with the conversion overlapped with the MFMAs and
# buffer loads (old vs new binary, alternated), the access-mix ceilings,
# the GEMM / block / item / e2e / parity / training tests, bench + profile
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04_v7
for v in old new2 old new2; do
  echo "== $v" >> gpurun_out/${T}_gemm_ab.txt
  timeout -k 10 120 tools/bin/gemm_ab_$v 204632 9 >> gpurun_out/${T}_gemm_ab.txt 2>&1 || exit $?
done
timeout -k 10 120 tools/bin/mix_bench 204632 7 > gpurun_out/${T}_mix_bench.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm_half.py tests/test_gpu_gemm.py tests/test_gpu_blocks.py tests/test_gpu_items.py tests/test_gpu_e2e.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_train.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-c5 --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
    -- python3 bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab > gpurun_out/${T}_prof.log 2>&1
rc=$?
cp gpurun_out/prof/bench_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv 2>/dev/null
python tools/step_sequence.py gpurun_out/prof/bench_kernel_trace.csv 10 > gpurun_out/${T}_step_sequence.txt 2>&1
rm -rf gpurun_out/prof
exit $rc
