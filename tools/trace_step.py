#!/usr/bin/env python
"""Per-step kernel-time breakdown and idle gaps from a rocprofv3 kernel trace
of bench.py (step boundary: the fused Adam kernel, 2 launches per step).

    python tools/trace_step.py gpurun_out/prof/*kernel_trace.csv [steps]"""
import collections
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "multi_tensor_apply" in r["Kernel_Name"]]
    a, b = adam[-(2 * S + 1)], adam[-1]
    seg = rows[a + 1:b + 1]
    t0, t1 = int(rows[a]["End_Timestamp"]), int(rows[b]["End_Timestamp"])
    cat = collections.defaultdict(lambda: [0.0, 0])
    for r in seg:
        n = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / S / 1e3
        if n.startswith("Cijk"):
            c = "hipBLASLt/rocBLAS GEMM"
        elif "k_gemm_nt" in n:
            c = "split-bf16 GEMM"
        elif "rocprim" in n:
            c = "rocprim (embedding plan)"
        elif "rb::" in n:
            m = re.search(r"(k_\w+)", n)
            c = m.group(1) if m else n[:40]
        else:
            c = "torch: " + re.sub(r"<.*", "", n.replace("void ", ""))[:50]
        cat[c][0] += d
        cat[c][1] += 1 / S
    gaps, prev = 0, t0
    for r in seg:
        s = int(r["Start_Timestamp"])
        if s > prev:
            gaps += s - prev
        prev = max(prev, int(r["End_Timestamp"]))
    print(f"wall/step {(t1 - t0) / S / 1e3:.1f} us, kernel sum {sum(v[0] for v in cat.values()):.1f}"
          f" us, idle {gaps / S / 1e3:.1f} us")
    for k, (us, n) in sorted(cat.items(), key=lambda kv: -kv[1][0]):
        print(f"{us:9.1f} us {n:6.1f}x  {k}")


if __name__ == "__main__":
    main()
