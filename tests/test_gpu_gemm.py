"""The split-operand projection GEMMs inside the encoder (f16x3,
csrc/gemm_half.hip; kernel-level accuracy against fp64 is in
tests/test_gpu_gemm_half.py): the whole training step against the torch
(hipBLASLt) path, the batched weight-image refresh and the image cache
across optimizer steps (RecBLR.py:162,165,167,213,214)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_split_path_in_the_encoder_matches_torch_path(cuda, monkeypatch, split_gemm_calls):
    """The whole training step with the f16x3 GEMMs against the torch
    (hipBLASLt) path: same loss and gradients within fp32 re-association.
    B = 256, L = 50 (ntok ~ 6.5k): every projection of the split arm runs
    rb_gemm_nt_h (asserted) and none of the torch arm does."""
    from datamining_recblr_amd import linear
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset

    cfg = dict(hidden_size=128, loss_type="CE", num_layers=2, dropout_prob=0.0, expand=2,
               d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
               MAX_ITEM_LIST_LENGTH=50)
    torch.manual_seed(0)
    model = RecBLR(cfg, SyntheticDataset(500)).to(cuda)
    B, L = 256, 50
    g = torch.Generator().manual_seed(1)
    lengths = torch.randint(1, L + 1, (B,), generator=g)
    seq = torch.randint(1, 500, (B, L), generator=g) * (torch.arange(L)[None] < lengths[:, None])
    inter = {"item_id_list": seq.to(cuda), "item_length": lengths.to(cuda),
             "item_id": torch.randint(1, 500, (B,), generator=g).to(cuda)}
    res = {}
    for on in (False, True):
        monkeypatch.setattr(linear, "_split_on", on)
        n0 = len(split_gemm_calls)
        model.zero_grad()
        loss = model.calculate_loss(inter)
        loss.backward()
        launched = len(split_gemm_calls) - n0
        if on:
            assert launched >= 16, split_gemm_calls
            assert any(c[0] >= 4096 for c in split_gemm_calls)
        else:
            assert launched == 0, split_gemm_calls
        res[on] = (loss.item(), {n: p.grad.clone() for n, p in model.named_parameters()
                                 if p.grad is not None})
    assert abs(res[True][0] - res[False][0]) < 1e-5
    for n, gr in res[False][1].items():
        err = (res[True][1][n] - gr).abs().max().item()
        assert err <= 1e-5 + 1e-4 * gr.abs().max().item(), (n, err)


def test_batched_weight_splits_equal_single(cuda):
    """rb_gemm_h_split_weights with several weights, both orientations, in one
    launch writes exactly the images it writes one weight at a time."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(3)
    ws = [torch.randn(n, k, generator=g).to(cuda) for n, k in ((512, 128), (256, 512), (128, 256))]
    jobs, refs = [], []
    for w in ws:
        for tr in (False, True):
            ref = kernels.gemm_h_weight(w, transpose=tr)
            jobs.append((w, tr, torch.empty_like(ref)))
            refs.append(ref)
    kernels.gemm_h_split_weights(jobs)
    for (_, _, wf), ref in zip(jobs, refs):
        assert torch.equal(wf.view(torch.int16), ref.view(torch.int16))


def test_split_cache_tracks_optimizer_steps(cuda):
    """Cached split images (refreshed in one launch after each optimizer step)
    give bit-identical training to splitting at every GEMM call."""
    from datamining_recblr_amd import linear
    from datamining_recblr_amd.distributed import synthetic_interaction
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset

    cfg = dict(hidden_size=64, loss_type="CE", num_layers=2, dropout_prob=0.0, expand=2,
               d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
               MAX_ITEM_LIST_LENGTH=50)
    batches = [synthetic_interaction(256, 50, 300, cuda, seed=s) for s in range(3)]
    runs = []
    for cache in (True, False):
        linear._cache_on = cache
        linear.invalidate_split_cache()
        torch.manual_seed(0)
        model = RecBLR(cfg, SyntheticDataset(300)).to(cuda).train()
        opt = torch.optim.Adam(model.parameters(), lr=1e-2, fused=True)
        losses = []
        for b in batches + batches:
            opt.zero_grad(set_to_none=True)
            loss = model.calculate_loss(b)
            loss.backward()
            opt.step()
            losses.append(loss.item())
        runs.append((losses, [p.detach().clone() for p in model.parameters()]))
    linear._cache_on = True
    assert runs[0][0] == runs[1][0]
    for a, b in zip(runs[0][1], runs[1][1]):
        assert torch.equal(a, b)
