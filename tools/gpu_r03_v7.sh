mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r03_v7_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r03_v7_pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_v7_smoke.log 2>&1
rc2=$?; tail -2 gpurun_out/r03_v7_smoke.log; exit $(( rc | rc2 ))
