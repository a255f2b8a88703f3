#!/usr/bin/env python
"""Effective shader clock per kernel from one rocprofv3 run with
`--pmc GRBM_GUI_ACTIVE --kernel-trace`: GRBM_GUI_ACTIVE (summed over the 8
XCDs) / 8 / the dispatch's duration (MI355X_MICROARCH.md, DVFS give-back:
reads high on dispatches shorter than ~0.3 ms).  Prints, per kernel with a
median dispatch >= 50 us, the dispatch count, median duration and median
clock.  Profiled runs hold lower clocks than unprofiled ones: compare kernels
within one run.

    python tools/pmc_clock.py <dir of the run's CSVs>"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from step_sequence import short  # noqa: E402


def main():
    d = sys.argv[1]
    gui = {}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                gui[r["Dispatch_Id"]] = gui.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    per = defaultdict(list)
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            g = gui.get(r["Dispatch_Id"])
            if g is None:
                continue
            ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            if ns > 0:
                per[short(r["Kernel_Name"])].append((ns / 1e3, g / 8 / ns))
    rows = []
    for k, v in per.items():
        us = statistics.median(x[0] for x in v)
        if us >= 50:
            rows.append((us, k, len(v), statistics.median(x[1] for x in v)))
    for us, k, n, ghz in sorted(rows, reverse=True):
        print(f"{k[:70]:70s} n={n:4d} median {us:8.1f} us  clock {ghz:5.2f} GHz")


if __name__ == "__main__":
    main()
