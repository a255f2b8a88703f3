#!/usr/bin/env python
"""Where the host spends the time before a launch that the GPU waited for:
from a rocprofv3 --kernel-trace --hip-trace run (CSV), for the timed-loop
step `first` (as tools/step_sequence.py counts steps) list every launch whose
idle gap before it exceeds `min_gap_us`, with the HIP API calls the host made
between the previous launch's API call and this one (name, duration) and the
host-side interval.

    python tools/host_gap.py <prefix> [first] [min_gap_us]
      (<prefix>_kernel_trace.csv and <prefix>_hip_api_trace.csv)"""
import collections
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from step_sequence import short  # noqa: E402


def main():
    pre = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    min_gap = float(sys.argv[3]) if len(sys.argv) > 3 else 30.0
    ks = list(csv.DictReader(open(pre + "_kernel_trace.csv")))
    api = list(csv.DictReader(open(pre + "_hip_api_trace.csv")))
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    api.sort(key=lambda r: int(r["Start_Timestamp"]))
    by_corr = {r["Correlation_Id"]: r for r in api}
    ends = [i for i, r in enumerate(ks) if "k_adam" in r["Kernel_Name"]
            or "multi_tensor_apply" in r["Kernel_Name"]]
    seg = ks[ends[first - 1] + 1:ends[first] + 1]
    t0 = int(ks[ends[first - 1]]["End_Timestamp"])
    print(f"# step {first}: {len(seg)} launches, {(int(seg[-1]['End_Timestamp']) - t0) / 1e3:.1f} us")
    # every HIP call the host made during the step's GPU window, by total time
    w0, w1 = t0, int(seg[-1]["End_Timestamp"])
    tot = collections.Counter()
    cnt = collections.Counter()
    longest = []
    for c in api:
        cs, ce = int(c["Start_Timestamp"]), int(c["End_Timestamp"])
        if w0 <= cs <= w1:
            tot[c["Function"]] += ce - cs
            cnt[c["Function"]] += 1
            longest.append((ce - cs, c["Function"], (cs - t0) / 1e3))
    print("# host HIP calls started inside the step's GPU window (total us, count):")
    for f, ns in tot.most_common(12):
        print(f"#   {f:40s} {ns / 1e3:9.1f} us  x{cnt[f]}")
    longest.sort(reverse=True)
    print("# longest single calls (us, function, start relative to the step):")
    for ns, f, at in longest[:8]:
        print(f"#   {ns / 1e3:9.1f}  {f}  at {at:.1f}")
    # where the host stands: each launch call's host time vs its kernel's start
    lag = []
    for r in seg:
        a = by_corr.get(r["Correlation_Id"])
        if a is not None:
            lag.append((int(r["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
    if lag:
        print(f"# launch call -> kernel start: min {min(lag):.1f} us, median "
              f"{sorted(lag)[len(lag) // 2]:.1f} us, max {max(lag):.1f} us (small: the GPU "
              f"waited for the host)")
    prev_end = t0
    prev_api = by_corr.get(ks[ends[first - 1]]["Correlation_Id"])
    starts = [int(r["Start_Timestamp"]) for r in api]
    import bisect
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        a = by_corr.get(r["Correlation_Id"])
        gap = (s - prev_end) / 1e3
        if gap >= min_gap and a is not None and prev_api is not None:
            h0, h1 = int(prev_api["End_Timestamp"]), int(a["Start_Timestamp"])
            print(f"\n{short(r['Kernel_Name'])}: GPU idle {gap:.1f} us before it; host "
                  f"{(h1 - h0) / 1e3:.1f} us from the previous launch call to this one; the "
                  f"launch call came {(int(a['Start_Timestamp']) - prev_end) / 1e3:+.1f} us "
                  f"after the previous kernel ended")
            i0, i1 = bisect.bisect_left(starts, h0), bisect.bisect_right(starts, h1)
            agg = collections.OrderedDict()
            for c in api[i0:i1]:
                d = agg.setdefault(c["Function"], [0, 0])
                d[0] += 1
                d[1] += int(c["End_Timestamp"]) - int(c["Start_Timestamp"])
            for f, (n, ns) in agg.items():
                print(f"    {f:40s} x{n:3d} {ns / 1e3:8.1f} us")
        prev_end = e
        if a is not None:
            prev_api = a


if __name__ == "__main__":
    main()
