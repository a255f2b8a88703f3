"""Train / evaluate RecBLR on a RecBole atomic .inter file (run.py's flow:
data preparation, fit with early stopping on valid NDCG@10, test metrics).

    python tools/train_real.py --inter dataset/amazon-beauty/amazon-beauty.inter
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/train_real.py --inter ...
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from datamining_recblr_amd.data import from_atomic_file  # noqa: E402
from datamining_recblr_amd.distributed import init_from_env  # noqa: E402
from datamining_recblr_amd.model import RecBLR  # noqa: E402
from datamining_recblr_amd.recbole_compat import SyntheticDataset  # noqa: E402
from datamining_recblr_amd.trainer import fit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--inter", required=True)
    ap.add_argument("--hidden", type=int, default=64)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--dropout", type=float, default=0.2)
    ap.add_argument("--max-len", type=int, default=200)
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--stopping-step", type=int, default=10)
    ap.add_argument("--seed", type=int, default=2020)
    a = ap.parse_args()
    env = init_from_env()
    dev = torch.device("cuda", env.local_rank)
    torch.cuda.set_device(dev)
    data = from_atomic_file(a.inter, max_len=a.max_len).to(dev)
    cfg = {"hidden_size": a.hidden, "loss_type": "CE", "num_layers": a.layers,
           "dropout_prob": a.dropout, "expand": 2, "d_conv": 4, "bd_lru_only": False,
           "disable_conv1d": False, "disable_ffn": False, "MAX_ITEM_LIST_LENGTH": a.max_len}
    torch.manual_seed(a.seed)
    model = RecBLR(cfg, SyntheticDataset(data.n_items, data.n_users)).to(dev)
    res = fit(model, data, env, epochs=a.epochs, batch_size=a.batch, lr=a.lr,
              stopping_step=a.stopping_step, seed=a.seed,
              log=lambda r: print(json.dumps(r), flush=True))
    if env.rank == 0:
        print(json.dumps({"best_valid_ndcg@10": res["best_valid"], "test": res["test"]}))


if __name__ == "__main__":
    main()
