mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o c5 \
    -- python3 tools/c5_step.py 4 > gpurun_out/c5_prof.log 2>&1
rc=$?
cp gpurun_out/prof/c5_kernel_stats.csv gpurun_out/c5_kernel_stats.csv 2>/dev/null
rm -rf gpurun_out/prof
exit $rc
