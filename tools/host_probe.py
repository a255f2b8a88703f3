#!/usr/bin/env python
"""Host-side cost of one training step of bench.py's workload: time to
enqueue a step (no synchronisation) against the step's GPU time, plus a
cProfile of the enqueue path.  If enqueue ~ GPU time the step is host-bound."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from datamining_recblr_amd.distributed import synthetic_interaction  # noqa: E402
from datamining_recblr_amd.model import RecBLR  # noqa: E402
from datamining_recblr_amd.recbole_compat import SyntheticDataset  # noqa: E402

dev = torch.device("cuda")
cfg = dict(hidden_size=128, loss_type="CE", num_layers=2, dropout_prob=0.2, expand=2, d_conv=4,
           bd_lru_only=False, disable_conv1d=False, disable_ffn=False, MAX_ITEM_LIST_LENGTH=200)
torch.manual_seed(2020)
model = RecBLR(cfg, SyntheticDataset(10544)).to(dev).train()
opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
batches = [synthetic_interaction(2048, 200, 10544, dev, seed=i) for i in range(4)]


def step(i):
    opt.zero_grad(set_to_none=True)
    loss = model.calculate_loss(batches[i % 4])
    loss.backward()
    opt.step()


for i in range(5):
    step(i)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(20):
    step(i)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"enqueue {1e3 * (t1 - t0) / 20:.3f} ms/step, total {1e3 * (t2 - t0) / 20:.3f} ms/step")
pr = cProfile.Profile()
torch.cuda.synchronize()
pr.enable()
for i in range(5):
    step(i)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
