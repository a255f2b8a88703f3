"""Shared inputs of tests/test_gpu_ddp.py and its rank processes
(tests/ddp_worker.py): the model config and the global batches."""
import torch

CFG = dict(hidden_size=128, loss_type="CE", num_layers=2, dropout_prob=0.0, expand=2,
           d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False)


def batches(global_batch, L, n_items, steps):
    """`steps` RecBole-shaped CPU batches (lengths ~U{1..L}, right-padded)."""
    out = []
    for s in range(steps):
        g = torch.Generator().manual_seed(100 + s)
        lengths = torch.randint(1, L + 1, (global_batch,), generator=g)
        seq = torch.randint(1, n_items, (global_batch, L), generator=g)
        seq = seq * (torch.arange(L)[None] < lengths[:, None])
        out.append({"item_id_list": seq, "item_length": lengths,
                    "item_id": torch.randint(1, n_items, (global_batch,), generator=g)})
    return out


def to_device(full, lo, hi, dev):
    """Rows [lo, hi) of a CPU batch on `dev`, host lengths attached."""
    from datamining_recblr_amd.model import attach_host_lengths

    shard = {k: v[lo:hi].to(dev) for k, v in full.items()}
    attach_host_lengths(shard["item_length"], full["item_length"][lo:hi])
    return shard
