"""The CE forward on the f16 pipe (rb_item_ce_fwd_h) alone at the bench's
scoring shape (B = 2048 rows, V = 10,544 items, d = 128): median of 50
HIP-event timings, plus an FNV-1a checksum of (loss, lse) so two builds can
be compared bit for bit.  python tools/ce_fwd_probe.py [B V d]"""
import sys

import torch

sys.path.insert(0, ".")
from datamining_recblr_amd import kernels  # noqa: E402


def main(B=2048, V=10544, d=128):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    seq = torch.randn(B, d, device=dev, generator=g)
    tab = torch.randn(V, d, device=dev, generator=g) * 0.1
    tgt = torch.randint(1, V, (B,), device=dev, generator=g)
    s_seq, s_tab = kernels.item_split_h(seq), kernels.item_split_h(tab)
    ts = []
    for i in range(60):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        loss, lse = kernels.item_ce_fwd_h(s_seq, s_tab, tgt)
        e1.record()
        torch.cuda.synchronize()
        if i >= 10:
            ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    h = 1469598103934665603
    for w in torch.cat([loss.view(1), lse]).view(torch.int32).cpu().tolist():
        h = ((h ^ (w & 0xffffffff)) * 1099511628211) & ((1 << 64) - 1)
    print(f"ce_fwd_h B={B} V={V} d={d}: median {ts[len(ts) // 2]:.1f} us, min {ts[0]:.1f} us, "
          f"loss {loss.item():.6f}, fnv {h:016x}", flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
