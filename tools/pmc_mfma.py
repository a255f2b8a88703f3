#!/usr/bin/env python
"""Per-kernel MFMA busy fraction and MFMA FLOPs from one rocprofv3 PMC pass:

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F32 \
        SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 \
        --output-format csv -d gpurun_out/pmc_mfma -o run \
        -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-full-tail
    python tools/pmc_mfma.py gpurun_out/pmc_mfma > profiles/rNN_pmc_mfma.json

MfmaUtil follows rocprofv3's derived metric on gfx950:
    sum(SQ_VALU_MFMA_BUSY_CYCLES) / (max(GRBM_GUI_ACTIVE) * SIMD_NUM)
(SIMD_NUM = 4 x 256 CUs); MFMA FLOPs = MOPS x 512 (rocprofv3's MfmaFlops*).
The counter CSV holds GRBM_GUI_ACTIVE summed over the 8 XCDs (a 740-us GEMM
reports 13.8 M cycles = 8 x 1.73 M at 2.4 GHz), so the per-XCD maximum the
derived metric wants is taken as that sum / 8.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMD_NUM = 1024
N_XCD = 8


def short(name):
    n = name.replace("void ", "").replace("rb::(anonymous namespace)::", "")
    return n.split("(")[0][:90]


def main():
    d = sys.argv[1]
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [(dispatch, value)]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            per[row["Kernel_Name"]][row["Counter_Name"]].append(
                (row.get("Dispatch_Id", ""), float(row["Counter_Value"])))
    out = {}
    for k, cs in per.items():
        def total(c):
            # values are per dispatch (already reduced over SEs/XCDs by rocprofv3)
            return sum(v for _, v in cs.get(c, []))
        n = max(len(cs.get("GRBM_GUI_ACTIVE", [])), 1)
        busy, act = total("SQ_VALU_MFMA_BUSY_CYCLES"), total("GRBM_GUI_ACTIVE")
        f32, bf16 = total("SQ_INSTS_VALU_MFMA_MOPS_F32"), total("SQ_INSTS_VALU_MFMA_MOPS_BF16")
        f16 = total("SQ_INSTS_VALU_MFMA_MOPS_F16")
        if f32 + bf16 + f16 == 0:
            continue
        out[short(k)] = {"dispatches": n,
                         "mfma_util": round(busy / (act / N_XCD * SIMD_NUM), 4) if act else None,
                         "mfma_flops_f32_per_dispatch": f32 * 512 / n,
                         "mfma_flops_bf16_per_dispatch": bf16 * 512 / n,
                         "mfma_flops_f16_per_dispatch": f16 * 512 / n,
                         "gui_active_cycles_per_xcd_per_dispatch": act / N_XCD / n,
                         "implied_us_at_2p4GHz": round(act / N_XCD / n / 2400.0, 1)}
    json.dump({"source": d, "formula": "MfmaUtil = sum(SQ_VALU_MFMA_BUSY_CYCLES) / "
               "(GRBM_GUI_ACTIVE_per_XCD * SIMD_NUM), SIMD_NUM = 1024, GRBM_GUI_ACTIVE_per_XCD = CSV sum / 8", "kernels":
               dict(sorted(out.items(), key=lambda kv: -(kv[1]["mfma_flops_f32_per_dispatch"]
                                                + kv[1]["mfma_flops_f16_per_dispatch"])))},
              sys.stdout, indent=1)


if __name__ == "__main__":
    main()
