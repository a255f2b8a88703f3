#!/usr/bin/env python
"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950: 3 + 2 of the 4 TCC slots).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py ...
    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/rNN_pmc_traffic.json

Counters are in KiB.  MI355X_MICROARCH.md (HBM/rocprofv3): on gfx950
FETCH_SIZE reports half the bytes of a wide (16-B/lane) coalesced streaming
read, WRITE_SIZE is exact for 16-B stores; other access widths must be
calibrated on a known byte count.  The calibration kernel is rb_scan_fwd in
bench.py's forward-only scan microbench (k_scan_rows_fwd<true>: float4 loads
and stores, algorithmic 2N*4 read + N*4 written): the printed
read_scale / write_scale are algorithmic / counted bytes for that kernel and
are applied to every kernel ("corrected" values).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    out = defaultdict(list)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            out[row["Kernel_Name"]].append((int(row["Grid_Size"]), float(row["Counter_Value"])))
    return out


def demangle(name):
    """rocprofv3 leaves some template instances mangled (_ZN2rb...)."""
    if not name.startswith("_Z"):
        return name
    import subprocess
    try:
        return subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt", name], capture_output=True,
                              text=True, check=True).stdout.strip() or name
    except (OSError, subprocess.SubprocessError):
        return name


def short(name):
    n = demangle(name).replace("void ", "").replace("rb::(anonymous namespace)::", "")
    return n.split("(")[0]


def modes(vals, tol=0.03):
    """[{"bytes": mean, "launches": n}] of the values grouped within tol."""
    out = []
    for v in sorted(vals):
        if out and abs(v - out[-1]["_ref"]) <= tol * max(out[-1]["_ref"], 1.0):
            out[-1]["_sum"] += v
            out[-1]["launches"] += 1
        else:
            out.append({"_ref": v, "_sum": v, "launches": 1})
    return [{"bytes": round(m["_sum"] / m["launches"]), "launches": m["launches"]} for m in out]


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    # calibration: the [2048, 256, 200] forward scan (largest grid of the kernel)
    cal_read = cal_write = None
    for name, vals in fetch.items():
        if "k_scan_rows_fwd" in name:
            grid, kib = max(vals)
            rows = grid // 64            # one wave per row
            T = int(os.environ.get("CAL_T", "200"))
            algo_r = 2 * rows * T * 4
            cal_read = algo_r / (kib * 1024)
            wv = write.get(name)
            if wv:
                algo_w = rows * T * 4
                cal_write = algo_w / (max(wv)[1] * 1024)
    res = {"calibration": {"kernel": "k_scan_rows_fwd<true> (float4 loads/stores)",
                           "read_scale": cal_read, "write_scale": cal_write,
                           "note": "algorithmic bytes / counted bytes on the calibration kernel"},
           "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        if not (name.startswith("void rb::") or name.startswith("rb::")
                or name.startswith("_ZN2rb")):
            continue
        fv = [v for _, v in fetch.get(name, [])]
        wv = [v for _, v in write.get(name, [])]
        # per launch, over the launches of the largest grid (the benchmark shape)
        fr = sorted(fetch.get(name, []))
        wr = sorted(write.get(name, []))
        gmax = max([g for g, _ in fr] + [g for g, _ in wr] + [0])
        fsel = [v for g, v in fr if g == gmax]
        wsel = [v for g, v in wr if g == gmax]
        f_b = 1024 * sum(fsel) / len(fsel) if fsel else None
        w_b = 1024 * sum(wsel) / len(wsel) if wsel else None
        res["kernels"][short(name)] = {
            "grid": gmax, "launches": len(fsel),
            "fetch_bytes_raw": f_b, "write_bytes_raw": w_b,
            "fetch_bytes": f_b * cal_read if (f_b and cal_read) else f_b,
            "write_bytes": w_b * cal_write if (w_b and cal_write) else w_b,
        }
        k = res["kernels"][short(name)]
        if k["fetch_bytes"] is not None and k["write_bytes"] is not None:
            k["traffic_bytes"] = k["fetch_bytes"] + k["write_bytes"]
        # launches of one kernel that move different byte counts at the same
        # grid (e.g. the LayerNorm forward in gather mode vs with a residual):
        # the distinct per-launch values, clustered within 3%, with counts
        k["fetch_modes"] = modes([v * 1024 * (cal_read or 1) for v in fsel])
        k["write_modes"] = modes([v * 1024 * (cal_write or 1) for v in wsel])
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
