"""Pieces of the CE backward on the f16 pipe (scoring._bwd_f16) at the bench
shape, HIP-event timed (median of 20): transposed probs, the NT product
ditems = P^T seq, the TN product dseq = P W (+ column sum), the row-group
maxima; against torch.mm on P."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from datamining_recblr_amd import kernels, scoring  # noqa: E402
from datamining_recblr_amd.linear import _tn_splits  # noqa: E402


def t(fn, reps=20):
    ts = []
    for i in range(reps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if i >= 3:
            ts.append(e0.elapsed_time(e1) * 1e3)
    return sorted(ts)[len(ts) // 2]


B, V, d = 2048, 10544, 128
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
seq = (0.3 * torch.randn(B, d, generator=g)).to(dev)
W = (0.3 * torch.randn(V, d, generator=g)).to(dev)
tgt = torch.randint(0, V, (B,), generator=g).to(dev)
ss, sw = kernels.item_split_h(seq), kernels.item_split_h(W)
_, lse = kernels.item_ce_fwd_h(ss, sw, tgt)
dl = torch.ones((), device=dev)
pt, gmax = kernels.item_ce_probs_h_t(ss, sw, tgt, lse, dl)
p = kernels.item_ce_probs_h(ss, sw, tgt, lse, dl)
img = kernels.gemm_h_weight(seq, transpose=True)
S = _tn_splits(dev, (B // 128) * (d // 128)) // 2
xm = scoring._group_max(W)
res = {
    "probs_h (P)": t(lambda: kernels.item_ce_probs_h(ss, sw, tgt, lse, dl)),
    "probs_h_t (P^T + group max)": t(lambda: kernels.item_ce_probs_h_t(ss, sw, tgt, lse, dl)),
    "seq^T image": t(lambda: kernels.gemm_h_weight(seq, transpose=True)),
    "NT ditems = P^T seq": t(lambda: kernels.gemm_nt_h(pt, img, d)),
    "group max of W": t(lambda: scoring._group_max(W)),
    f"TN dseq partials (S={S})": t(lambda: kernels.gemm_tn_h(pt, W, gmax, xm, S)),
    "colsum": t(lambda: kernels.colsum(torch.empty(S, B * d, device=dev))),
    "torch.mm P W": t(lambda: torch.mm(p, W)),
    "torch.mm P^T seq": t(lambda: torch.mm(p.t(), seq)),
}
for k, v in res.items():
    print(f"{k:32s} {v:8.1f} us")

# the both-layouts plan: ditems = TN over the batch rows of P [B, Vp] (Vp = V
# rounded to 256), dseq = TN over the item rows of P^T, each + column sum
Vp = (V + 255) // 256 * 256
pbuf = torch.zeros(B, Vp, device=dev)
kernels.item_ce_probs_h(ss, sw, tgt, lse, dl, out=pbuf[:, :V])
bmax = scoring._group_max(pbuf)
smax = scoring._group_max(seq)
res2 = {}
for S1 in (8, 16):
    res2[f"TN ditems on P (S={S1})"] = t(lambda: kernels.gemm_tn_h(pbuf, seq, bmax, smax, S1))
    res2[f"colsum [{S1}, Vp*d]"] = t(lambda: kernels.colsum(torch.empty(S1, Vp * d, device=dev)))
for S2 in (16, 32, 64):
    res2[f"TN dseq on P^T (S={S2})"] = t(lambda: kernels.gemm_tn_h(pt, W, gmax, xm, S2))
    res2[f"colsum [{S2}, B*d]"] = t(lambda: kernels.colsum(torch.empty(S2, B * d, device=dev)))
for k, v in res2.items():
    print(f"{k:32s} {v:8.1f} us")
# accuracy of the two products against fp64 on the same P
ref_items = (p.double().t() @ seq.double())
ref_seq = (p.double() @ W.double())
di = kernels.colsum(kernels.gemm_tn_h(pbuf, seq, bmax, smax, 8).view(8, -1)).view(Vp, d)[:V]
ds = kernels.colsum(kernels.gemm_tn_h(pt, W, gmax, xm, 32).view(32, -1)).view(B, d)
for nm, a, r in (("ditems", di, ref_items), ("dseq", ds, ref_seq)):
    e = ((a.double() - r).abs().max() / r.abs().max()).item()
    et = (((p.t() @ seq if nm == "ditems" else p @ W).double() - r).abs().max() / r.abs().max()).item()
    print(f"{nm}: rel err {e:.3e} (torch fp32 {et:.3e})")
