"""Does the host run ahead of the GPU in the bench's loop, and where does it
block?  The bench's step (B=2048, L=200, d=128, packed, native Adam) run 40
times without synchronizing: the host time at which each step's launches
were queued, then a cProfile of 20 more steps (top functions by own time).
python tools/host_lead_probe.py"""
import cProfile
import json
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from datamining_recblr_amd.distributed import synthetic_interaction  # noqa: E402
from datamining_recblr_amd.model import RecBLR  # noqa: E402
from datamining_recblr_amd.optim import Adam  # noqa: E402
from datamining_recblr_amd.recbole_compat import SyntheticDataset  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    cfg = dict(hidden_size=128, loss_type="CE", num_layers=2, dropout_prob=0.2, expand=2,
               d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
               MAX_ITEM_LIST_LENGTH=200)
    torch.manual_seed(2020)
    model = RecBLR(cfg, SyntheticDataset(10544)).to(dev).train()
    opt = Adam(model.parameters(), lr=1e-3)
    batches = [synthetic_interaction(2048, 200, 10544, dev, seed=i) for i in range(4)]

    def step(i):
        opt.zero_grad(set_to_none=True)
        loss = model.calculate_loss(batches[i % 4])
        loss.backward()
        opt.step()
        return loss

    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    marks = []
    for i in range(40):
        step(i)
        marks.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    d = [round(1e3 * (b - a), 3) for a, b in zip([0.0] + marks[:-1], marks)]
    print(json.dumps({"host_ms_per_step": d, "gpu_ms_per_step": round(1e3 * total / 40, 3),
                      "host_done_ms": round(1e3 * marks[-1], 2), "total_ms": round(1e3 * total, 2)}),
          flush=True)
    # The same steps with the host certainly ahead: 4 steps queued behind
    # ~50 ms of busy GEMMs (busy, so the clocks stay up; the pinned rings hold
    # 4), timed by events between the GEMMs' end and the 4th step's end.
    # Equal to the steady-state time per step = no host-induced GPU idle.
    pre = []
    big = torch.randn(8192, 8192, device=dev)
    for trial in range(4):
        for i in range(4):
            step(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(6):
            torch.mm(big, big)
        e0.record()
        for i in range(4):
            step(trial * 4 + i)
        e1.record()
        queued_ahead = not e0.query()   # the spin still running: all 4 steps queued before it ended
        torch.cuda.synchronize()
        pre.append((round(e0.elapsed_time(e1) / 4, 3), queued_ahead))
    t0e, t1e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    for i in range(8):
        step(i)
    t0e.record()
    for i in range(16):
        step(i)
    t1e.record()
    torch.cuda.synchronize()
    print(json.dumps({"prequeued_ms_per_step": pre,
                      "steady_ms_per_step": round(t0e.elapsed_time(t1e) / 16, 3)}), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(20):
        step(i)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
