"""world_size-2 gloo test of the batch-DP path used by bench.py --gpus N:
env-driven init, the DDP LossModule wrapper, per-rank sharding and the
max-over-ranks timer.  The encoder itself needs a GPU, so the CPU stand-in
model here exercises the same wrapper and all-reduce plumbing."""
import os
import socket

import torch
import torch.multiprocessing as mp
from torch import nn


class TinyRec(nn.Module):
    """calculate_loss-shaped model: embedding -> mean -> CE over all items."""

    def __init__(self, n_items=30, d=8):
        super().__init__()
        self.item_embedding = nn.Embedding(n_items, d)
        self.proj = nn.Linear(d, d)

    def calculate_loss(self, inter):
        h = self.proj(self.item_embedding(inter["item_id_list"]).mean(1))
        return nn.functional.cross_entropy(h @ self.item_embedding.weight.t(), inter["item_id"])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, queue):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from datamining_recblr_amd.distributed import (init_from_env, max_over_ranks, shard_range,
                                                   synthetic_interaction, wrap_ddp)

    env = init_from_env(backend="gloo")
    torch.manual_seed(0)
    model = TinyRec()
    step = wrap_ddp(model, env)
    full = synthetic_interaction(12, 6, 30, "cpu", seed=3)
    lo, hi = shard_range(12, env.rank, env.world_size)
    shard = {k: v[lo:hi] for k, v in full.items()}
    loss = step(shard)
    loss.backward()
    t = max_over_ranks(float(rank + 1), env)
    grads = {n: p.grad.detach().numpy().copy() for n, p in model.named_parameters()}
    queue.put((rank, t, grads))
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_gloo_world2_matches_full_batch():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from datamining_recblr_amd.distributed import synthetic_interaction

    torch.manual_seed(0)
    ref = TinyRec()
    ref.calculate_loss(synthetic_interaction(12, 6, 30, "cpu", seed=3)).backward()
    for rank, tmax, grads in results:
        assert tmax == float(world)
        for n, p in ref.named_parameters():
            torch.testing.assert_close(torch.from_numpy(grads[n]), p.grad, atol=1e-6, rtol=1e-5)


def _seed_worker(rank, world, port, queue):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from datamining_recblr_amd.blocks import draw_seed
    from datamining_recblr_amd.distributed import init_from_env

    init_from_env(backend="gloo")
    torch.manual_seed(2020)          # every rank seeds alike (RecBole's config seed)
    queue.put((rank, [draw_seed() for _ in range(3)]))
    dist.barrier()
    dist.destroy_process_group()


def test_dropout_keys_differ_across_ranks():
    """The Philox dropout key folds in the rank: equal generator seeds on two
    ranks still give different masks for their different batch shards; rank 0
    keeps the single-process stream."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_seed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from datamining_recblr_amd.blocks import draw_seed

    torch.manual_seed(2020)
    single = [draw_seed() for _ in range(3)]
    assert got[0] == single
    assert all(a != b for a, b in zip(got[0], got[1]))
    assert all(0 <= s < 2 ** 62 for s in got[1])


class ParamShapedRec(nn.Module):
    """RecBLR's parameters (d = 128, n_items = 10,544, two layers: the bench's
    model, built on the CPU) behind a CPU loss that uses each of them once in
    module order, so the backward finishes them in reverse order as the real
    step does — the item table last."""

    def __init__(self):
        super().__init__()
        from datamining_recblr_amd.model import RecBLR
        from datamining_recblr_amd.recbole_compat import SyntheticDataset
        self.inner = RecBLR(dict(hidden_size=128, loss_type="CE", num_layers=2, dropout_prob=0.2,
                                 expand=2, d_conv=4, bd_lru_only=False, disable_conv1d=False,
                                 disable_ffn=False, MAX_ITEM_LIST_LENGTH=200),
                            SyntheticDataset(10544))

    def calculate_loss(self, inter):
        s = inter["item_id"].float().mean()
        h = torch.zeros(())
        for i, p in enumerate(self.inner.parameters()):
            h = h * 0.5 + (p * (s + i)).square().mean()
        return h


def _bucket_worker(rank, world, port, queue):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from datamining_recblr_amd.distributed import init_from_env, wrap_ddp

    env = init_from_env(backend="gloo")
    torch.manual_seed(0)
    model = ParamShapedRec()
    step = wrap_ddp(model, env)
    full = {"item_id": torch.arange(1, 9)}
    shard = {"item_id": full["item_id"][4 * rank:4 * rank + 4]}
    for _ in range(3):   # static_graph: buckets are rebuilt at the third forward
        model.zero_grad(set_to_none=True)
        step(shard).backward()
    buckets = step.reducer._get_zeros_like_grad_buckets()
    sizes = [b.buffer().numel() * 4 for b in buckets]
    emb = model.inner.item_embedding.weight
    last = [any(p.shape == emb.shape for p in b.parameters()) for b in buckets]
    grads = {n: p.grad.detach().numpy().copy() for n, p in model.named_parameters()}
    queue.put((rank, sizes, last, grads))
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_buckets_overlap_the_backward():
    """wrap_ddp's bucket size gives the bench's model >= 3 gradient buckets
    (all-reduces that can start during the backward), the item table, whose
    gradient is finished last, in the last one; gradients equal the
    single-process ones averaged."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    ref = ParamShapedRec()
    ga = {}
    for r in range(world):
        ref.zero_grad(set_to_none=True)
        ref.calculate_loss({"item_id": torch.arange(1, 9)[4 * r:4 * r + 4]}).backward()
        for n, p in ref.named_parameters():
            ga[n] = ga.get(n, 0) + p.grad / world
    for rank, sizes, last, grads in results:
        assert len(sizes) >= 3, sizes
        assert sum(sizes) == 4 * sum(p.numel() for p in ref.parameters())
        assert last == [False] * (len(sizes) - 1) + [True], (sizes, last)
        for n in ga:
            torch.testing.assert_close(torch.from_numpy(grads[n]), ga[n], atol=1e-6, rtol=1e-5)
