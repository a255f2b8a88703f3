"""GPU tests of the split-bf16 fp32 GEMM (csrc/gemm_split.hip, rb_gemm_nt):
F.linear's forward and input-gradient products (RecBLR.py:162,165,167,213,
214) against an fp64 product, with the error held to the level of torch's own
fp32 GEMM (hipBLASLt) on the same data — the claim is fp32-level accuracy,
not bf16."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel_err(y, ref):
    return ((y.double() - ref).abs().max() / ref.abs().max()).item()


@pytest.mark.parametrize("M,K,N", [(4096, 128, 512), (5000, 256, 512), (4097, 512, 128),
                                   (8192, 256, 128), (300, 128, 256), (1, 32, 128),
                                   (257, 512, 384)])
@pytest.mark.parametrize("bias", [False, True])
def test_forward_matches_fp64_at_fp32_accuracy(cuda, M, K, N, bias):
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(M + K + N)
    x = torch.randn(M, K, generator=g).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = torch.randn(N, generator=g).to(cuda) if bias else None
    y = kernels.gemm_nt(x, kernels.gemm_split_weight(w), N, bias=b)
    ref = x.double() @ w.double().t()
    if bias:
        ref = ref + b.double()
    yt = torch.addmm(b, x, w.t()) if bias else x @ w.t()
    e_split, e_torch = _rel_err(y, ref), _rel_err(yt, ref)
    # fp32-level: a few ulps relative to the output scale, on a par with hipBLASLt
    assert e_split < 2e-6, e_split
    assert e_split < 4 * max(e_torch, 1e-7), (e_split, e_torch)


@pytest.mark.parametrize("M,N,K", [(4096, 512, 128), (4100, 256, 512), (1024, 128, 256)])
def test_input_gradient_and_accumulate(cuda, M, N, K):
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(7 * M + N)
    dy = torch.randn(M, N, generator=g).to(cuda)
    w = (torch.randn(N, K, generator=g) / N ** 0.5).to(cuda)
    wt = kernels.gemm_split_weight(w, transpose=True)
    dx = kernels.gemm_nt(dy, wt, K)
    ref = dy.double() @ w.double()
    assert _rel_err(dx, ref) < 2e-6
    base = torch.randn(M, K, generator=g).to(cuda)
    out = base.clone()
    kernels.gemm_nt(dy, wt, K, out=out, accumulate=True)
    assert _rel_err(out, base.double() + ref) < 2e-6


def test_row_strided_operand_and_output(cuda):
    """A as a column slice of a wider activation (the x half of xz), out as a
    row-strided view — the layouts the encoder hands over."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(3)
    big = torch.randn(4096, 512, generator=g).to(cuda)
    x = big[:, 256:]                      # row stride 512, 16-B aligned
    w = (torch.randn(256, 256, generator=g) / 16).to(cuda)
    outbig = torch.zeros(4096, 384, device=cuda)
    out = outbig[:, :256]
    kernels.gemm_nt(x, kernels.gemm_split_weight(w), 256, out=out)
    ref = x.double() @ w.double().t()
    assert _rel_err(out, ref) < 2e-6
    assert outbig[:, 256:].abs().max().item() == 0.0


def test_split_path_in_the_encoder_matches_torch_path(cuda, monkeypatch, split_gemm_calls):
    """The whole training step with the split-bf16 GEMM against the torch
    (hipBLASLt) path: same loss and gradients within fp32 re-association.
    B = 256, L = 50 (ntok ~ 6.5k, above SPLIT_MIN_ROWS) and the threshold at 0
    in the split arm, so every projection of that arm runs rb_gemm_nt (asserted)
    and none of the torch arm does."""
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
        monkeypatch.setattr(linear, "SPLIT_MIN_ROWS", 0 if on else 4096)
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
    """rb_gemm_split_weights (several weights, both orientations, one launch)
    writes exactly the images rb_gemm_split_weight writes one at a time."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(3)
    ws = [torch.randn(n, k, generator=g).to(cuda) for n, k in ((512, 128), (256, 512), (128, 256))]
    jobs, refs = [], []
    for w in ws:
        for tr in (False, True):
            ref = kernels.gemm_split_weight(w, transpose=tr)
            jobs.append((w, tr, torch.empty_like(ref)))
            refs.append(ref)
    kernels.gemm_split_weights(jobs)
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
