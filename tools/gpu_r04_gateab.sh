# Gates-GEMM epilogue ablations at the bench shape (tools/gate_ab.hip built
# by tools/gate_ab_variants.py), alternated; then the gate tests again
mkdir -p gpurun_out
O=gpurun_out/r04_gate_ab.txt
for v in full rgonly noload nowait nomath full rgonly noload nowait nomath; do
  timeout -k 10 120 tools/bin/gate_ab_$v 2048 9 >> $O 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_gate_gemm.py > gpurun_out/r04_gate_pytest_gate2.log 2>&1 || exit $?
