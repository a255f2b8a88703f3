"""One rank of tests/test_gpu_ddp.py (started as a child process, never
imported by pytest): RecBLR wrapped by distributed.wrap_ddp, trained for a
few Adam steps on this rank's shard of a fixed global batch; writes the loss
and every parameter gradient of every step to OUT (a tensor-only .pt).

argv: OUT STEPS GLOBAL_BATCH L N_ITEMS.  Env: RANK, WORLD_SIZE, LOCAL_RANK,
MASTER_ADDR, MASTER_PORT (torchrun's), RB_DDP_BACKEND (default gloo).
Every rank runs on cuda:0 (the test box has one GPU)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out, steps, gb, L, n_items = sys.argv[1], *map(int, sys.argv[2:6])
    import torch
    import torch.distributed as dist

    from datamining_recblr_amd.distributed import init_from_env, shard_range, wrap_ddp
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset
    from tests.ddp_common import CFG, batches, to_device

    from datamining_recblr_amd import kernels

    tn_rows = []                       # M of every rb_gemm_tn_h launch (weight gradients)
    _tn = kernels.gemm_tn_h

    def counted(dy, x, *a, **kw):
        tn_rows.append(dy.shape[0])
        return _tn(dy, x, *a, **kw)

    kernels.gemm_tn_h = counted
    env = init_from_env(backend=os.environ.get("RB_DDP_BACKEND", "gloo"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(2020)
    model = RecBLR(dict(CFG, MAX_ITEM_LIST_LENGTH=L), SyntheticDataset(n_items)).to(dev).train()
    step_mod = wrap_ddp(model, env)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
    lo, hi = shard_range(gb, env.rank, env.world_size)
    rec = {}
    for i, full in enumerate(batches(gb, L, n_items, steps)):
        shard = to_device(full, lo, hi, dev)
        opt.zero_grad(set_to_none=True)
        loss = step_mod(shard)
        loss.backward()
        rec[f"loss.{i}"] = loss.detach().cpu().reshape(1)
        for n, p in model.named_parameters():
            rec[f"grad.{i}.{n}"] = p.grad.detach().cpu().clone()
        opt.step()
    for n, p in model.named_parameters():
        rec[f"param.{n}"] = p.detach().cpu().clone()
    rec["dist"] = torch.tensor([int(dist.is_initialized()), env.world_size])
    rec["tn_rows"] = torch.tensor(tn_rows, dtype=torch.int64)
    torch.save(rec, out)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
