"""Softmax-CE over the item table, fwd+bwd: torch (materialised logits) vs the
fused MFMA forward with the two backward strategies.  Median of 20 after 3
warm-ups, HIP events; peak memory from torch's allocator.

    python tools/ce_bench.py [B V d ...]
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from datamining_recblr_amd import scoring  # noqa: E402


def run(fn, reps=20):
    ts = []
    for i in range(reps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if i >= 3:
            ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    shapes = [(2048, 10544, 128), (2048, 262144, 128), (1024, 10544, 256), (2048, 10544, 64)]
    if len(sys.argv) > 3:
        a = list(map(int, sys.argv[1:]))
        shapes = [tuple(a[i:i + 3]) for i in range(0, len(a), 3)]
    dev = torch.device("cuda:0")
    for B, V, d in shapes:
        g = torch.Generator(device="cpu").manual_seed(0)
        seq = (0.3 * torch.randn(B, d, generator=g)).to(dev).requires_grad_()
        W = (0.3 * torch.randn(V, d, generator=g)).to(dev).requires_grad_()
        tgt = torch.randint(0, V, (B,), generator=g).to(dev)

        def torch_path():
            F.cross_entropy(seq @ W.t(), tgt).backward()

        def ours(mode):
            def f():
                scoring.CE_BACKWARD = mode
                scoring.item_cross_entropy(seq, W, tgt).backward()
            return f

        res = {}
        for name, fn in (("torch", torch_path), ("fused_fwd+slices", ours("slices")),
                         ("fused_fwd+fused_bwd", ours("fused"))):
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats()
            base = torch.cuda.memory_allocated()
            us = run(fn)
            peak = (torch.cuda.max_memory_allocated() - base) / 2 ** 20
            res[name] = us
            print(f"B={B} V={V} d={d} {name:22s} {us:9.1f} us  "
                  f"{6 * B * V * d / us / 1e6:6.1f} TF/s(3 GEMM-equiv)  peak +{peak:8.1f} MiB",
                  flush=True)
            seq.grad = W.grad = None


if __name__ == "__main__":
    main()
