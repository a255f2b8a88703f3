#!/usr/bin/env python
"""SQ counters of the NT GEMM per gemmbench_h shape (tools/pmc_gemm_h.sh
passes): each counter summed over a shape's 12 timed dispatches, printed per
k-step of one workgroup where that reads better.

    python tools/pmc_gemm_sq.py gpurun_out/pmc_gh1 gpurun_out/pmc_gh2
"""
import csv
import glob
import os
import sys
from collections import defaultdict

SHAPES = ["in.fwd", "in.dX", "gates.fwd", "gates.dX", "out.fwd", "out.dX", "w2.fwd", "w2.dX"]


def main():
    per = defaultdict(lambda: defaultdict(float))   # dispatch -> counter -> value
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                if "gemm_nt_h" not in r["Kernel_Name"]:
                    continue
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(per)
    n = len(ids) // len(SHAPES)
    counters = sorted({c for v in per.values() for c in v})
    print("shape      " + " ".join(f"{c[3:]:>18s}" for c in counters))
    for i, nm in enumerate(SHAPES):
        sel = ids[i * n:(i + 1) * n]
        vals = [sum(per[k][c] for k in sel) / len(sel) for c in counters]
        print(f"{nm:10s} " + " ".join(f"{v:18.4g}" for v in vals))


if __name__ == "__main__":
    main()
