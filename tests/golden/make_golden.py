#!/usr/bin/env python
"""Generate the golden vectors by RUNNING THE REFERENCE in this container.

    python tests/golden/make_golden.py        # ~5 min on 8 CPU cores

* parallel_scan.py is executed through Triton's CPU interpreter
  (TRITON_INTERPRET=1), i.e. the reference's own forward_scan/backward_scan
  kernels and Scan autograd glue;
* RecBLR.py is imported with a minimal recbole stand-in
  (tests/golden/recbole_stub, our own code) because recbole==1.2.0 is not
  installable offline; causal_conv1d is absent, so the reference takes its
  F.conv1d fallback (RecBLR.py:184-185).

Only inputs/outputs are written (tests/golden/*.pt, plain tensor dicts loaded
with weights_only=True); no reference source travels with the repo.  The
reference tree (/root/reference) is needed only to REGENERATE the fixtures.
"""
from __future__ import annotations

import math
import os
import sys

os.environ["TRITON_INTERPRET"] = "1"
sys.dont_write_bytecode = True
REF = os.environ.get("RECBLR_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "recbole_stub"), REF]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import RecBLR as ref_model  # noqa: E402  (the reference module)
from parallel_scan import parallel_scan as ref_scan  # noqa: E402

assert os.path.dirname(os.path.abspath(ref_model.__file__)) == os.path.abspath(REF), ref_model.__file__

torch.set_num_threads(8)


class _Dataset:
    def __init__(self, n_items):
        self.n_items = n_items

    def num(self, field):
        assert field == "item_id"
        return self.n_items


def _lambda(C):
    lo = ref_model.softplus_inverse(torch.tensor(-math.log(0.9))).item()
    hi = ref_model.softplus_inverse(torch.tensor(-math.log(0.999))).item()
    return torch.linspace(lo, hi, C)


def scan_cases():
    out = []
    for seed, shape in enumerate([(2, 3, 8), (4, 16, 64), (2, 4, 256), (1, 2, 2048), (3, 5, 1),
                                  (2, 2, 4)]):
        g = torch.Generator().manual_seed(seed)
        B, C, T = shape
        r = torch.randn(B, C, T, generator=g)
        gates = torch.exp(-F.softplus(_lambda(C))[None, :, None] * torch.sigmoid(r))
        tokens = torch.randn(B, C, T, generator=g)
        grad = torch.randn(B, C, T, generator=g)
        ga = gates.clone().requires_grad_()
        to = tokens.clone().requires_grad_()
        states = ref_scan(ga, to)
        states.backward(grad)
        out.append(dict(gates=gates, tokens=tokens, grad=grad, states=states.detach(),
                        d_gates=ga.grad, d_tokens=to.grad))
        print("scan", shape, flush=True)
    return out


def grl_cases():
    out = []
    specs = [  # d, L, B, disable_conv1d, kernel
        (16, 50, 3, False, 4), (16, 64, 2, False, 4), (16, 200, 2, False, 4),
        (64, 50, 2, False, 4), (16, 1, 2, False, 4), (16, 3, 2, False, 4),
        (16, 50, 2, True, 4), (16, 33, 2, False, 2), (8, 100, 2, False, 4)]
    for seed, (d, L, B, dc, k) in enumerate(specs):
        torch.manual_seed(100 + seed)
        layer = ref_model.GatedRecurrentLayer(d_model=d, kernel_size=k, disable_conv1d=dc)
        with torch.no_grad():  # non-trivial Lambda (the init is a plain linspace)
            layer.Lambda.add_(0.3 * torch.randn_like(layer.Lambda))
        x = torch.randn(B, L, d)
        gy = torch.randn(B, L, d)
        xi = x.clone().requires_grad_()
        y = layer(xi)
        (y * gy).sum().backward()
        out.append(dict(
            d=d, L=L, B=B, disable_conv1d=dc, kernel_size=k,
            params={n: p.detach().clone() for n, p in layer.named_parameters()},
            x=x, gy=gy, y=y.detach(), dx=xi.grad,
            grads={n: p.grad.clone() for n, p in layer.named_parameters()
                   if p.grad is not None}))
        print("grl", d, L, B, dc, k, flush=True)
    return out


def model_cases():
    out = []
    base = dict(hidden_size=32, loss_type="CE", num_layers=2, dropout_prob=0.2, expand=2,
                d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
                MAX_ITEM_LIST_LENGTH=50)
    specs = [
        dict(), dict(loss_type="BPR", hidden_size=16, MAX_ITEM_LIST_LENGTH=20),
        dict(hidden_size=16, disable_conv1d=True), dict(hidden_size=16, disable_ffn=True),
        dict(hidden_size=16, bd_lru_only=True, num_layers=1),
        dict(hidden_size=16, MAX_ITEM_LIST_LENGTH=64),
    ]
    n_items = 64
    for ci, spec in enumerate(specs):
        cfg = dict(base, **spec)
        torch.manual_seed(2020)
        model = ref_model.RecBLR(cfg, _Dataset(n_items))
        init_state = {k: v.detach().clone() for k, v in model.state_dict().items()}
        model.eval()
        B, L = 4, cfg["MAX_ITEM_LIST_LENGTH"]
        g = torch.Generator().manual_seed(ci)
        lengths = torch.tensor([1, L, max(1, L // 3), max(1, L - 7)])
        seq = torch.randint(1, n_items, (B, L), generator=g)
        seq = seq * (torch.arange(L)[None, :] < lengths[:, None])   # RecBole right-pads with 0
        pos = torch.randint(1, n_items, (B,), generator=g)
        neg = torch.randint(1, n_items, (B,), generator=g)
        inter = {"item_id_list": seq, "item_length": lengths, "item_id": pos, "neg_item_id": neg}
        loss = model.calculate_loss(inter)
        loss.backward()
        with torch.no_grad():
            seq_out = model.forward(seq, lengths)
            scores = seq_out @ model.item_embedding.weight.t()   # == full_sort_predict
            pred = (seq_out * model.item_embedding(pos)).sum(1)  # == predict
        out.append(dict(cfg=cfg, n_items=n_items, init_state=init_state, item_seq=seq,
                        item_seq_len=lengths, pos_items=pos, neg_items=neg, loss=loss.detach(),
                        seq_output=seq_out, full_sort=scores, predict=pred,
                        grads={n: p.grad.clone() for n, p in model.named_parameters()
                               if p.grad is not None}))
        print("model", spec, float(loss), flush=True)
    return out


def main():
    torch.save({"cases": scan_cases()}, os.path.join(HERE, "scan_golden.pt"))
    torch.save({"cases": grl_cases()}, os.path.join(HERE, "grl_golden.pt"))
    torch.save({"cases": model_cases()}, os.path.join(HERE, "model_golden.pt"))
    for f in ("scan_golden.pt", "grl_golden.pt", "model_golden.pt"):
        print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
