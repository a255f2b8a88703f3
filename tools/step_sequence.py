#!/usr/bin/env python
"""One training step's kernel sequence from a rocprofv3 kernel trace of
bench.py: every launch in issue order with its duration, the idle gap before
it and its predecessor, plus the step's launch count and the time in launches
under 20 us.  Steps end at the optimizer kernel (torch's fused Adam:
multi_tensor_apply; rb_adam_step: k_adam); the median-length step of the last
`steps` is printed — or of the `steps` steps starting at step `first`
(0-based over the whole trace: bench.py's timed loop starts after its
warmup steps, before the host-enqueue, breakdown and variant passes).

    python tools/step_sequence.py <kernel_trace.csv> [steps] [first] > out.txt"""
import csv
import re
import sys


def short(name: str) -> str:
    n = name.replace("void ", "")
    if n.startswith("Cijk"):
        return "hipBLASLt:" + n[:40]
    m = re.search(r"rb::\(anonymous namespace\)::(\w+)(<[^(]*>)?", n)
    if m:
        return m.group(1) + (m.group(2) or "")[:60]
    m = re.search(r"(k_\w+)", n)
    if m:
        return m.group(1)
    return re.sub(r"<.*", "", n)[:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    first = int(sys.argv[3]) if len(sys.argv) > 3 else None
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows)
            if "multi_tensor_apply" in r["Kernel_Name"] or "k_adam" in r["Kernel_Name"]]
    # a fused torch Adam may be several launches per step: keep the last of a run
    ends = [e for k, e in enumerate(ends) if k + 1 == len(ends) or ends[k + 1] != e + 1]
    steps = []
    # step k spans (ends[k-1], ends[k]]; the first step (k = 0) has no
    # predecessor end and is never selected
    pairs = (list(zip(ends[first - 1:first + S - 1], ends[first:first + S])) if first
             else list(zip(ends[-(S + 1):-1], ends[-S:])))
    for a, b in pairs:
        seg = rows[a + 1:b + 1]
        t0 = int(rows[a]["End_Timestamp"])
        t1 = int(rows[b]["End_Timestamp"])
        steps.append((t1 - t0, seg, t0))
    steps.sort(key=lambda x: x[0])
    wall, seg, t0 = steps[len(steps) // 2]
    print(f"# median of {len(steps)} steps: {wall / 1e3:.1f} us wall, {len(seg)} launches")
    small = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in seg
                if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) < 20000)
    nsmall = sum(1 for r in seg if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) < 20000)
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    print(f"# kernel time {busy / 1e3:.1f} us; launches under 20 us: {nsmall}, "
          f"{small / 1e3:.1f} us; idle {(wall - busy) / 1e3:.1f} us")
    print(f"{'#':>4} {'start_us':>9} {'dur_us':>8} {'gap_us':>7}  kernel  (predecessor)")
    prev_end, prev = t0, "-"
    for k, r in enumerate(seg):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        nm = short(r["Kernel_Name"])
        print(f"{k:4d} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {(s - prev_end) / 1e3:7.1f}  "
              f"{nm}  ({prev})")
        prev_end, prev = e, nm


if __name__ == "__main__":
    main()
