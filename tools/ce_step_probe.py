"""The CE backward's two weight-gradient products (scoring._bwd_f16) timed in
the training step and again, in isolation, on the very operands the step
passed them (captured), plus the same isolated calls on operands with the
step's shapes but uniform random values: is the in-step slowness the data,
the splits, or the step's context?  One line per measurement."""
import sys
import time

import torch

sys.path.insert(0, ".")
from datamining_recblr_amd import kernels  # noqa: E402
from datamining_recblr_amd.distributed import synthetic_interaction  # noqa: E402
from datamining_recblr_amd.model import RecBLR  # noqa: E402
from datamining_recblr_amd.recbole_compat import SyntheticDataset  # noqa: E402


def ev_time(fn, reps=9):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda:0")
    B, L, N_ITEMS = 2048, 200, 10544
    cfg = dict(hidden_size=128, loss_type="CE", num_layers=2, dropout_prob=0.2, expand=2,
               d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
               MAX_ITEM_LIST_LENGTH=L)
    torch.manual_seed(2020)
    model = RecBLR(cfg, SyntheticDataset(N_ITEMS)).to(dev).train()
    inter = synthetic_interaction(B, L, N_ITEMS, dev, seed=0)
    calls = []
    orig = kernels.gemm_tn_h

    def rec(dy, x, ymax, xmax, splits):
        big = dy.shape[0] in (B, N_ITEMS) and dy.shape[1] in (B, (N_ITEMS + 255) // 256 * 256)
        if big:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = orig(dy, x, ymax, xmax, splits)
            e1.record()
            calls.append(((dy, x, ymax, xmax, splits), e0, e1))
            return out
        return orig(dy, x, ymax, xmax, splits)

    kernels.gemm_tn_h = rec
    for step in range(4):
        calls.clear()
        model.zero_grad(set_to_none=True)
        loss = model.calculate_loss(inter)
        loss.backward()
        torch.cuda.synchronize()
        for (a, e0, e1) in calls:
            print(f"step {step}: in-step gemm_tn_h dy{tuple(a[0].shape)} S={a[4]}: "
                  f"{e0.elapsed_time(e1) * 1e3:.1f} us", flush=True)
    kernels.gemm_tn_h = orig
    for (a, _, _) in calls:
        dy, x, ymax, xmax, S = a
        t = ev_time(lambda: orig(dy, x, ymax, xmax, S))
        print(f"isolated, captured operands dy{tuple(dy.shape)} S={S}: {t:.1f} us", flush=True)
        for S2 in (8, 16, 32, 64):
            if dy.shape[0] // S2 >= 32:
                t = ev_time(lambda: orig(dy, x, ymax, xmax, S2))
                print(f"   S={S2}: {t:.1f} us", flush=True)
        r = torch.rand_like(dy) * 1e-3
        rmax = torch.full_like(ymax, 1e-3)
        t = ev_time(lambda: orig(r, x, rmax, xmax, S))
        print(f"isolated, uniform random dy{tuple(dy.shape)} S={S}: {t:.1f} us", flush=True)
        # the captured operand's column spread inside 256-row chunks
        ch = dy[: dy.shape[0] // 256 * 256].view(-1, 256, dy.shape[1]).abs()
        cm = ch.amax(1)
        chunk = cm.amax(1, keepdim=True)
        frac = ((cm > 0) & (cm < chunk * 2.0 ** -16)).float().mean().item()
        print(f"   columns below 2^-16 of their chunk max: {frac:.4f}", flush=True)


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"done in {time.time() - t0:.1f} s")
