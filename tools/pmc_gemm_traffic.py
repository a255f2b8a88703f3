#!/usr/bin/env python
"""Summarise tools/pmc_gemm_traffic.sh: HBM bytes per k_gemm_nt_h dispatch,
in gemmbench_h's shape order (12 timed launches per shape after the sampled
check's launch), against each shape's algorithmic bytes (A read once +
output written once).  FETCH_SIZE x 2 (gfx950 counts half of a wide
streaming read, MI355X_MICROARCH.md), WRITE_SIZE as counted; KiB.

    python tools/pmc_gemm_traffic.py gpurun_out <variant> [M]
"""
import csv
import glob
import os
import sys

SHAPES = [("in.fwd", 128, 512), ("in.dX", 512, 128), ("gates.fwd", 256, 512),
          ("gates.dX", 512, 256), ("out.fwd", 256, 128), ("out.dX", 128, 256),
          ("w2.fwd", 512, 128), ("w2.dX", 128, 512)]


def load(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and "gemm_nt_h" in r["Kernel_Name"]:
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"]) * 1024))
    rows.sort()
    return [v for _, v in rows]


def main():
    out, v = sys.argv[1], sys.argv[2]
    M = int(sys.argv[3]) if len(sys.argv) > 3 else 204632
    fe = load(os.path.join(out, f"pmcg_{v}_FETCH_SIZE"), "FETCH_SIZE")
    wr = load(os.path.join(out, f"pmcg_{v}_WRITE_SIZE"), "WRITE_SIZE")
    per = len(fe) // len(SHAPES)
    print(f"variant {v}: {len(fe)} dispatches, {per} per shape")
    for i, (nm, R, C) in enumerate(SHAPES):
        f = sorted(fe[i * per:(i + 1) * per])[per // 2] * 2
        w = sorted(wr[i * per:(i + 1) * per])[per // 2]
        ar, aw = 4.0 * M * R, 4.0 * M * C
        print(f"{nm:10s} read {f / 1e6:8.1f} MB ({f / ar:4.2f}x A)  write {w / 1e6:7.1f} MB "
              f"({w / aw:4.2f}x out)")


if __name__ == "__main__":
    main()
