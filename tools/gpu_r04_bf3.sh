# per-shape bf16 GEMM timings (own vs torch) and the NT kernel's SQ counters
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04_bf3
timeout -k 10 300 python -u tools/bf16_gemm_probe.py > gpurun_out/${T}_shapes.txt 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES \
    --output-format csv -d gpurun_out/pmc_bf -o run -- python3 tools/bf16_gemm_probe.py 524288 > gpurun_out/${T}_pmc.log 2>&1 || exit $?
python - <<'PY' > gpurun_out/${T}_pmc.txt 2>&1
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_bf/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f[0])):
    k = r["Kernel_Name"][:60]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    if "gemm" in k or "Cijk" in k:
        print(k, {c: f"{x:.3e}" for c, x in sorted(v.items())})
PY
rm -rf gpurun_out/pmc_bf
