# Round-4 closing evidence: the whole GPU suite, smoke, the default bench
# line, the rocprof kernel summary + one step's kernel sequence, and the PMC
# passes (HBM traffic, MFMA busy) whose summaries the bench line cites
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04_final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
    -- python3 bench.py --no-cpu-baseline --no-full-tail --no-c5 --no-ddp-ab > gpurun_out/${T}_prof.log 2>&1 || exit $?
cp gpurun_out/prof/bench_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv
python tools/step_sequence.py gpurun_out/prof/bench_kernel_trace.csv 10 > gpurun_out/${T}_step_sequence.txt 2>&1
rm -rf gpurun_out/prof
bash tools/pmc_all.sh || exit $?
cp gpurun_out/pmc_traffic.json gpurun_out/${T}_pmc_traffic.json
cp gpurun_out/pmc_mfma.json gpurun_out/${T}_pmc_mfma.json
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_mfma
# the bench line cites the newest profiles/*_pmc_*.json: this lease's
cp gpurun_out/${T}_pmc_traffic.json profiles/${T}_pmc_traffic.json
cp gpurun_out/${T}_pmc_mfma.json profiles/${T}_pmc_mfma.json
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.log 2>&1
