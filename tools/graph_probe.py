"""Does capturing the training step as a HIP graph shrink the gaps between
launches?    The bench's step (B=2048, L=200, d=128,
n_items 10,544, packed, dropout 0.2, native Adam) timed two ways on one
lease, alternated:

  eager   - the bench's loop (host queues launches ahead of the GPU);
  graph   - the same step captured once per batch with torch.cuda.graph and
            replayed (one launch of the whole DAG; dropout seeds are frozen
            into the capture, so this is a timing probe, not a training mode).

Prints one JSON line.  Usage: python tools/graph_probe.py [--steps 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from datamining_recblr_amd.distributed import synthetic_interaction  # noqa: E402
from datamining_recblr_amd.model import RecBLR  # noqa: E402
from datamining_recblr_amd.optim import Adam  # noqa: E402
from datamining_recblr_amd.recbole_compat import SyntheticDataset  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = dict(hidden_size=128, loss_type="CE", num_layers=2, dropout_prob=0.2, expand=2,
               d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
               MAX_ITEM_LIST_LENGTH=200)
    torch.manual_seed(2020)
    model = RecBLR(cfg, SyntheticDataset(10544)).to(dev).train()
    opt = Adam(model.parameters(), lr=1e-3)
    # one batch for both loops: the capture bakes the packed layout's host
    # staging slot into the graph, whose content must stay this batch's
    batches = [synthetic_interaction(2048, 200, 10544, dev, seed=0)] * 4

    def step(b):
        opt.zero_grad(set_to_none=False)
        loss = model.calculate_loss(b)
        loss.backward()
        opt.step()
        return loss

    for i in range(8):
        step(batches[i % 4])
    torch.cuda.synchronize()

    graphs = []
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for b in batches:
            for _ in range(2):
                step(b)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step(batches[0])
    graphs = [g] * 4
    torch.cuda.synchronize()

    def time_eager():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(batches[i % 4])
        torch.cuda.synchronize()
        return 1000.0 * (time.perf_counter() - t0) / args.steps

    def time_graph():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            graphs[i % 4].replay()
        torch.cuda.synchronize()
        return 1000.0 * (time.perf_counter() - t0) / args.steps

    res = {"eager": [], "graph": []}
    for _ in range(args.rounds):
        res["eager"].append(round(time_eager(), 4))
        res["graph"].append(round(time_graph(), 4))
    print(json.dumps({"probe": "graph_vs_eager", "ms_per_step": res,
                      "eager_min": min(res["eager"]), "graph_min": min(res["graph"]),
                      "note": "graph replay of the whole step (frozen dropout seeds) vs the "
                              "eager loop, alternated on one lease"}), flush=True)


if __name__ == "__main__":
    main()
