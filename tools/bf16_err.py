#!/usr/bin/env python
"""Measure the GatedRecurrentLayer bf16-storage error against the fp32 oracle
(the quantity tests/test_gpu_bf16.py::test_grl_bf16_vs_oracle bounds), over
several seeds, so the test's tolerance rests on measured numbers.  Prints one
JSON line: per shape, the max over seeds of max|a - ref| / max|ref| for y, dx
and every parameter gradient."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import recblr_oracle as orc  # noqa: E402
from datamining_recblr_amd.model import GatedRecurrentLayer  # noqa: E402

BF = torch.bfloat16


def one(B, L, d, seed, dev):
    torch.manual_seed(seed)
    layer = GatedRecurrentLayer(d_model=d).to(dev)
    g = torch.Generator().manual_seed(seed + 6)
    x32 = torch.randn(B, L, d, generator=g).to(BF).float()
    gy = torch.randn(B, L, d, generator=g).to(BF).float()
    x = x32.to(dev).to(BF).requires_grad_()
    y = layer(x)
    (y.float() * gy.to(dev)).sum().backward()
    params = {k: v.detach().cpu().requires_grad_() for k, v in layer.state_dict().items()}
    xs = x32.clone().requires_grad_()
    ys = orc.grl_forward(params, "", xs)
    (ys * gy).sum().backward()

    def rel(a, b):
        return ((a.float().cpu() - b).abs().max() / b.abs().max()).item()

    out = {"y": rel(y.detach(), ys.detach()), "dx": rel(x.grad, xs.grad)}
    for n, p in layer.named_parameters():
        out["d" + n] = rel(p.grad, params[n].grad)
    return out


def main():
    dev = torch.device("cuda:0")
    res = {}
    for B, L, d in ((3, 50, 64), (2, 2048, 256)):
        worst = {}
        for seed in range(5, 10):
            for k, v in one(B, L, d, seed, dev).items():
                worst[k] = max(worst.get(k, 0.0), v)
        res[f"{B}x{L}x{d}"] = {k: float(f"{v:.3e}") for k, v in worst.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
