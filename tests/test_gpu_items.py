"""GPU parity of the item-scoring kernels (csrc/item_scores.hip) against plain
torch fp64 compositions of the reference's ops: logits = seq @ W^T and
nn.CrossEntropyLoss (RecBLR.py:100-102), full_sort_predict's scores
(RecBLR.py:114-122) and the target rank that RecBole's full-sort evaluator
and run_with_unseen.py:229-265 reduce them to.

Tolerances: the kernels sum each dot product as one k-ordered fp32 fma chain
(error <= ~d * 2^-24 * sum|a b|), torch's fp64 reference is exact to fp32
precision; 2e-5 relative on losses and normwise 2e-5 on gradients."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [(1, 1, 16), (5, 7, 32), (33, 64, 64), (64, 1000, 128), (300, 10544, 128),
          (37, 515, 256), (130, 97, 64), (2048, 10544, 128)]


def _data(B, V, d, cuda, seed=0, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed * 1000 + B * 7 + V * 3 + d)
    seq = (scale * torch.randn(B, d, generator=g)).to(cuda)
    W = (scale * torch.randn(V, d, generator=g)).to(cuda)
    tgt = torch.randint(0, V, (B,), generator=g).to(cuda)
    return seq, W, tgt


def normwise(a, b, tol, what):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    err = (a - b).norm() / max(b.norm().item(), 1e-30)
    assert err < tol, f"{what}: normwise err {err:.3e}"


@pytest.mark.parametrize("B,V,d", SHAPES)
def test_item_scores_match_matmul(cuda, B, V, d):
    from datamining_recblr_amd import kernels

    seq, W, _ = _data(B, V, d, cuda)
    out = kernels.item_scores(seq, W)
    ref = seq.double() @ W.double().t()
    bound = (seq.double().abs() @ W.double().abs().t()) * (d * 2.0 ** -23)
    assert ((out.double() - ref).abs() <= bound + 1e-30).all()


@pytest.mark.parametrize("B,V,d", SHAPES)
def test_item_rank_exact_against_scores(cuda, B, V, d):
    """n_greater / n_equal recomputed from the score kernel's output: the
    target-score dot product replays the MFMA chain, so counts are exact."""
    from datamining_recblr_amd import kernels

    seq, W, tgt = _data(B, V, d, cuda, seed=1)
    scores = kernels.item_scores(seq, W)
    gt, eq = kernels.item_rank(seq, W, tgt, first_item=1)
    ts = scores.gather(1, tgt[:, None])
    cols = torch.arange(V, device=cuda)[None, :]
    ok = (cols >= 1) & (cols != tgt[:, None])
    assert torch.equal(gt, ((scores > ts) & ok).sum(1))
    assert torch.equal(eq, ((scores == ts) & ok).sum(1))


def test_item_rank_ties_and_invalid_targets(cuda):
    from datamining_recblr_amd import kernels

    seq, W, tgt = _data(40, 300, 64, cuda, seed=2)
    W[100:110] = W[5]            # ten exact copies of item 5
    tgt[:8] = 5
    tgt[8] = 300                 # out of range
    tgt[9] = -1
    gt, eq = kernels.item_rank(seq, W, tgt, first_item=1)
    assert (eq[:8] == 10).all()
    assert gt[8] == -1 and gt[9] == -1
    scores = seq.double() @ W.double().t()
    ref_gt = ((scores[:8] > scores[:8, 5:6]) &
              (torch.arange(300, device=cuda)[None, :] >= 1)).sum(1)
    # fp32 vs fp64 ordering can only differ for near-ties, absent here
    assert torch.equal(gt[:8], ref_gt.to(gt.device))
    # first_item = 0 counts the padding item too
    gt0, _ = kernels.item_rank(seq, W, tgt, first_item=0)
    assert (gt0[:8] >= gt[:8]).all() and (gt0[:8] - gt[:8] <= 1).all()


@pytest.mark.parametrize("pipe", ["f16", "f32"])
@pytest.mark.parametrize("B,V,d", SHAPES)
def test_item_ce_matches_torch(cuda, monkeypatch, B, V, d, pipe):
    from datamining_recblr_amd import scoring
    from datamining_recblr_amd.scoring import item_cross_entropy

    monkeypatch.setattr(scoring, "CE_PIPE", pipe)
    seq, W, tgt = _data(B, V, d, cuda, seed=3, scale=0.5)
    s1 = seq.clone().requires_grad_()
    w1 = W.clone().requires_grad_()
    loss = item_cross_entropy(s1, w1, tgt)
    (2.5 * loss).backward()
    s2 = seq.double().requires_grad_()
    w2 = W.double().requires_grad_()
    ref = F.cross_entropy(s2 @ w2.t(), tgt)
    (2.5 * ref).backward()
    assert abs(loss.item() - ref.item()) <= 2e-5 * max(1.0, abs(ref.item()))
    normwise(s1.grad, s2.grad, 2e-5, "dseq")
    normwise(w1.grad, w2.grad, 2e-5, "ditems")


def test_item_ce_lse_and_large_logits(cuda):
    """Logits of magnitude ~100 (online log-sum-exp must not overflow)."""
    from datamining_recblr_amd import kernels

    seq, W, tgt = _data(96, 5000, 128, cuda, seed=4, scale=1.0)
    loss, lse = kernels.item_ce_fwd(seq, W, tgt)
    logits = seq.double() @ W.double().t()
    assert logits.abs().max() > 40
    ref_lse = torch.logsumexp(logits, 1)
    assert torch.allclose(lse.double(), ref_lse, rtol=2e-6, atol=2e-5)
    ref = F.cross_entropy(logits, tgt)
    assert abs(loss.item() - ref.item()) <= 2e-5 * abs(ref.item())


def test_item_ce_deterministic_and_partial_grads(cuda):
    from datamining_recblr_amd import kernels

    seq, W, tgt = _data(513, 2049, 64, cuda, seed=5, scale=0.3)
    l1, lse1 = kernels.item_ce_fwd(seq, W, tgt)
    l2, lse2 = kernels.item_ce_fwd(seq, W, tgt)
    assert torch.equal(l1, l2) and torch.equal(lse1, lse2)
    dl = torch.ones((), device=cuda)
    a1, b1 = kernels.item_ce_bwd(seq, W, tgt, lse1, dl)
    a2, b2 = kernels.item_ce_bwd(seq, W, tgt, lse1, dl)
    assert torch.equal(a1, a2) and torch.equal(b1, b2)
    a3, n3 = kernels.item_ce_bwd(seq, W, tgt, lse1, dl, want_items=False)
    n4, b4 = kernels.item_ce_bwd(seq, W, tgt, lse1, dl, want_seq=False)
    assert n3 is None and n4 is None
    assert torch.equal(a3, a1) and torch.equal(b4, b1)


def test_item_ce_invalid_target_is_nan(cuda):
    from datamining_recblr_amd import kernels

    seq, W, tgt = _data(8, 50, 32, cuda, seed=6)
    tgt[3] = 50
    loss, _ = kernels.item_ce_fwd(seq, W, tgt)
    assert torch.isnan(loss)


def test_model_full_sort_rank_and_predict(cuda):
    """RecBLR.full_sort_rank agrees with ranking full_sort_predict's scores."""
    from datamining_recblr_amd.distributed import synthetic_interaction
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset
    from datamining_recblr_amd.scoring import rank_metrics

    cfg = {"hidden_size": 64, "loss_type": "CE", "num_layers": 2, "dropout_prob": 0.2,
           "expand": 2, "d_conv": 4, "bd_lru_only": False, "disable_conv1d": False,
           "disable_ffn": False, "MAX_ITEM_LIST_LENGTH": 50}
    torch.manual_seed(0)
    model = RecBLR(cfg, SyntheticDataset(3000)).to(cuda).eval()
    inter = synthetic_interaction(257, 50, 3000, cuda, seed=7)
    with torch.no_grad():
        scores = model.full_sort_predict(inter)
        gt, eq = model.full_sort_rank(inter)
    ref = model.forward(inter["item_id_list"], inter["item_length"]).detach()
    normwise(scores, ref @ model.item_embedding.weight.detach().t(), 1e-6, "scores")
    t = inter["item_id"]
    masked = scores.clone()
    masked[:, 0] = -float("inf")
    ts = scores.gather(1, t[:, None])
    others = torch.ones_like(masked, dtype=torch.bool)
    others[torch.arange(257), t] = False
    assert torch.equal(gt, ((masked > ts) & others).sum(1))
    # RecBole-style top-k metrics from the full score matrix
    topk = masked.topk(20, dim=1).indices
    pos = (topk == t[:, None]).float()
    hit10 = pos[:, :10].sum(1).mean().item()
    m = rank_metrics(gt, eq, topk=(10, 20))
    assert abs(m["hit@10"] - hit10) < 1e-9
    ndcg20 = (pos / torch.log2(torch.arange(2, 22, device=cuda).float())).sum(1).mean().item()
    assert abs(m["ndcg@20"] - ndcg20) < 1e-6


@pytest.mark.parametrize("mode", ["slices", "fused"])
@pytest.mark.parametrize("B,V,d,slice_bytes", [(300, 10544, 128, 1 << 30), (64, 1000, 64, 64 * 4 * 96),
                                               (37, 515, 256, 37 * 4 * 64), (5, 7, 32, 1 << 30)])
def test_item_ce_backward_modes(cuda, monkeypatch, mode, B, V, d, slice_bytes):
    """Both backward strategies (item slices + library GEMMs, and the fully
    fused MFMA backward) against torch fp64, including multi-slice tables."""
    from datamining_recblr_amd import scoring

    monkeypatch.setattr(scoring, "CE_BACKWARD", mode)
    monkeypatch.setattr(scoring, "PROBS_SLICE_BYTES", slice_bytes)
    seq, W, tgt = _data(B, V, d, cuda, seed=8, scale=0.5)
    s1 = seq.clone().requires_grad_()
    w1 = W.clone().requires_grad_()
    (0.7 * scoring.item_cross_entropy(s1, w1, tgt)).backward()
    s2 = seq.double().requires_grad_()
    w2 = W.double().requires_grad_()
    (0.7 * F.cross_entropy(s2 @ w2.t(), tgt)).backward()
    normwise(s1.grad, s2.grad, 2e-5, "dseq")
    normwise(w1.grad, w2.grad, 2e-5, "ditems")


def test_item_ce_probs_slice_offsets(cuda):
    from datamining_recblr_amd import kernels

    seq, W, tgt = _data(50, 700, 64, cuda, seed=9)
    _, lse = kernels.item_ce_fwd(seq, W, tgt)
    dl = torch.full((), 2.0, device=cuda)
    full = kernels.item_ce_probs(seq, W, tgt, lse, dl)
    logits = seq.double() @ W.double().t()
    ref = (torch.softmax(logits, 1) - F.one_hot(tgt, 700).double()) * 2.0 / 50
    assert (full.double() - ref).abs().max() < 1e-6
    out = torch.full((50, 1000), 7.0, device=cuda)
    part = kernels.item_ce_probs(seq, W[300:600], tgt, lse, dl, item_offset=300, out=out[:, 100:400])
    assert torch.equal(part, full[:, 300:600])
    assert (out[:, :100] == 7).all() and (out[:, 400:] == 7).all()


# ---- the f16 pipe (two-part split operands, csrc/item_scores.hip) -----------------
# Scores there are x0.y0 + x0.y1 + x1.y0 of 11+11-bit parts of power-of-two
# scaled rows, accumulated in fp32: error <= ~(d * 2^-24 + 2^-21) * sum|a b|,
# the fp32 kernels' bound up to the dropped x1.y1 term — the same test
# tolerances as the fp32 pipe.


def _split_ref(x):
    """(x0, x1, e) of rb_item_split_h, restated with numpy on the host (exact
    power-of-two scaling in float64, RNE fp16 casts with subnormals)."""
    import numpy as np

    xn = x.cpu().numpy().astype(np.float64)
    m = np.abs(xn).max(1)
    e = np.where(m > 0, np.frexp(m)[1], 0).astype(np.int32)
    sv = (xn * np.exp2(14.0 - e)[:, None]).astype(np.float32)   # exact shift
    x0 = sv.astype(np.float16)
    x1 = (sv - x0.astype(np.float32)).astype(np.float16)
    dev = x.device
    return (torch.from_numpy(x0).to(dev), torch.from_numpy(x1).to(dev),
            torch.from_numpy(e).to(dev))


@pytest.mark.parametrize("n,d", [(1, 16), (37, 32), (300, 64), (1000, 128), (5, 256),
                                 (10544, 128), (64, 256)])
def test_item_split_h_planes(cuda, n, d):
    from datamining_recblr_amd import kernels

    g = torch.Generator(device="cpu").manual_seed(n + d)
    x = torch.randn(n, d, generator=g) * torch.exp2(torch.randint(-60, 60, (n, 1), generator=g).float())
    x[0, : d // 2] = 0.0
    if n > 2:
        x[2] = 0.0                      # an all-zero row
    x = x.to(cuda)
    sp = kernels.item_split_h(x)
    x0, x1, e = _split_ref(x)
    assert torch.equal(sp.exps, e)
    assert torch.equal(sp.img[:, :d], x0) and torch.equal(sp.img[:, d:], x1)
    back = torch.ldexp(sp.img[:, :d].double() + sp.img[:, d:].double(),
                       (sp.exps - 14)[:, None].double())
    rel = ((back - x.double()).abs().amax(1) / x.double().abs().amax(1).clamp_min(1e-300))
    assert (rel <= 2.0 ** -21).all()
    # with the 32-row group maxima (rb_item_split_h's group_max): the same
    # planes and exponents, and rb_group_absmax's values bit for bit
    sg = kernels.item_split_h(x, group_max=True)
    assert torch.equal(sg.img, sp.img) and torch.equal(sg.exps, sp.exps)
    assert torch.equal(sg.gmax, kernels.group_absmax(x))


@pytest.mark.parametrize("B,V,d", [(1, 1, 16), (33, 64, 64), (300, 10544, 128), (37, 515, 256),
                                   (2048, 10544, 128)])
def test_item_ce_f16_kernels_vs_fp64(cuda, B, V, d):
    """lse, loss and P on split images against fp64 (logits up to ~40 at d = 128)."""
    from datamining_recblr_amd import kernels

    seq_s, W_s, tgt = _data(B, V, d, cuda, seed=11, scale=1.0)
    logits = seq_s.double() @ W_s.double().t()
    ss, sw = kernels.item_split_h(seq_s), kernels.item_split_h(W_s)
    loss, lse = kernels.item_ce_fwd_h(ss, sw, tgt)
    ref_lse = torch.logsumexp(logits, 1)
    assert torch.allclose(lse.double(), ref_lse, rtol=2e-6, atol=2e-5)
    ref = F.cross_entropy(logits, tgt)
    assert abs(loss.item() - ref.item()) <= 2e-5 * max(1.0, abs(ref.item()))
    dl = torch.full((), 1.5, device=cuda)
    p = kernels.item_ce_probs_h(ss, sw, tgt, lse, dl)
    pref = (torch.softmax(logits, 1) - F.one_hot(tgt, V).double()) * 1.5 / B
    assert (p.double() - pref).abs().max() <= 2e-5 * 1.5 / B
    # deterministic
    loss2, lse2 = kernels.item_ce_fwd_h(ss, sw, tgt)
    assert torch.equal(loss, loss2) and torch.equal(lse, lse2)


def test_item_ce_f16_row_scales(cuda):
    """seq rows 2^k and item rows 2^-k (every exponent path), logits moderate:
    per-row scales make each row's relative accuracy independent of k."""
    from datamining_recblr_amd import kernels

    B, V, d = 64, 300, 64
    seq, W, tgt = _data(B, V, d, cuda, seed=12, scale=0.5)
    k = torch.randint(-60, 60, (1,)).item()
    seq_s = torch.ldexp(seq, torch.full((B, 1), float(k), device=cuda))
    W_s = torch.ldexp(W, torch.full((V, 1), float(-k), device=cuda))
    seq_s[5] = 0.0                                  # a zero row: logits 0
    logits = seq_s.double() @ W_s.double().t()
    loss, lse = kernels.item_ce_fwd_h(kernels.item_split_h(seq_s), kernels.item_split_h(W_s), tgt)
    assert torch.allclose(lse.double(), torch.logsumexp(logits, 1), rtol=2e-6, atol=2e-5)
    assert abs(loss.item() - F.cross_entropy(logits, tgt).item()) <= 2e-5


def test_item_ce_f16_probs_slices_and_invalid_target(cuda):
    from datamining_recblr_amd import kernels

    seq, W, tgt = _data(50, 700, 64, cuda, seed=13)
    ss, sw = kernels.item_split_h(seq), kernels.item_split_h(W)
    _, lse = kernels.item_ce_fwd_h(ss, sw, tgt)
    dl = torch.full((), 2.0, device=cuda)
    full = kernels.item_ce_probs_h(ss, sw, tgt, lse, dl)
    out = torch.full((50, 1000), 7.0, device=cuda)
    part = kernels.item_ce_probs_h(ss, sw.rows(300, 600), tgt, lse, dl, item_offset=300,
                                   out=out[:, 100:400])
    assert torch.equal(part, full[:, 300:600])
    assert (out[:, :100] == 7).all() and (out[:, 400:] == 7).all()
    tgt[3] = 700
    loss, _ = kernels.item_ce_fwd_h(ss, sw, tgt)
    assert torch.isnan(loss)


def test_item_ce_f16_engaged_in_training_loss(cuda):
    """The model's CE (calculate_loss) runs the f16 kernels by default."""
    from datamining_recblr_amd import kernels
    from datamining_recblr_amd.distributed import synthetic_interaction
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset

    cfg = {"hidden_size": 64, "loss_type": "CE", "num_layers": 1, "dropout_prob": 0.0,
           "expand": 2, "d_conv": 4, "bd_lru_only": False, "disable_conv1d": False,
           "disable_ffn": False, "MAX_ITEM_LIST_LENGTH": 20}
    model = RecBLR(cfg, SyntheticDataset(500)).to(cuda)
    inter = synthetic_interaction(16, 20, 500, cuda, seed=3)
    with kernels.kernel_timing() as t:
        model.calculate_loss(inter).backward()
    names = {r[0] for r in t.records}
    assert {"rb_item_split_h", "rb_item_ce_fwd_h", "rb_item_ce_probs_h"} <= names, names


def test_item_ce_f16_probs_transposed(cuda):
    """rb_item_ce_probs_h_t: P^T bit-identical to the row-major kernel's P,
    partial batch tile included, and the exact max |P| of every 32-item group."""
    from datamining_recblr_amd import kernels

    seq, W, tgt = _data(200, 1000, 128, cuda, seed=14)
    ss, sw = kernels.item_split_h(seq), kernels.item_split_h(W)
    _, lse = kernels.item_ce_fwd_h(ss, sw, tgt)
    dl = torch.full((), 1.5, device=cuda)
    p = kernels.item_ce_probs_h(ss, sw, tgt, lse, dl)
    pt, gmax = kernels.item_ce_probs_h_t(ss, sw, tgt, lse, dl)
    assert torch.equal(pt, p.t())
    want = torch.nn.functional.pad(p.abs().amax(0), (0, (-1000) % 32)).view(-1, 32).amax(1)
    assert torch.equal(gmax, want)
    # a slice of the table
    pt2, g2 = kernels.item_ce_probs_h_t(ss, sw.rows(320, 1000), tgt, lse, dl, item_offset=320)
    assert torch.equal(pt2, p[:, 320:].t())
    assert torch.equal(g2, want[10:])


def test_item_ce_f16_probs_both_layouts(cuda):
    """rb_item_ce_probs_h_both: P (zero-padded columns) and P^T bit-identical
    to the one-layout kernels, the 32-item group maxima equal to
    rb_item_ce_probs_h_t's and the 32-row group maxima exact, partial batch
    tile included; rb_group_absmax exact."""
    from datamining_recblr_amd import kernels

    seq, W, tgt = _data(200, 1000, 128, cuda, seed=16)
    ss, sw = kernels.item_split_h(seq), kernels.item_split_h(W)
    _, lse = kernels.item_ce_fwd_h(ss, sw, tgt)
    dl = torch.full((), 0.8, device=cuda)
    p_ref = kernels.item_ce_probs_h(ss, sw, tgt, lse, dl)
    pt_ref, g_ref = kernels.item_ce_probs_h_t(ss, sw, tgt, lse, dl)
    p, pt, bmax, gmax = kernels.item_ce_probs_h_both(ss, sw, tgt, lse, dl, pad_to=256)
    assert p.shape == (200, 1024) and torch.equal(p[:, :1000], p_ref)
    assert not p[:, 1000:].any()
    assert torch.equal(pt, pt_ref) and torch.equal(gmax, g_ref)
    want = torch.nn.functional.pad(p_ref.abs().amax(1), (0, (-200) % 32)).view(-1, 32).amax(1)
    assert torch.equal(bmax, want)
    x = torch.randn(1000, 96, device=cuda)
    want_x = torch.nn.functional.pad(x.abs().amax(1), (0, (-1000) % 32)).view(-1, 32).amax(1)
    assert torch.equal(kernels.group_absmax(x), want_x)
    assert torch.equal(kernels.group_absmax(x[:, 1:95]),
                       torch.nn.functional.pad(x[:, 1:95].abs().amax(1), (0, 24)).view(-1, 32).amax(1))


@pytest.mark.parametrize("B,V,slice_bytes,on", [(2048, 10544, 1 << 30, True),
                                                (512, 1000, 1 << 30, True),
                                                (256, 515, 256 * 4 * 96, False),
                                                (128, 33, 1 << 30, False)])
def test_item_ce_f16_grads_vs_fp64(cuda, monkeypatch, B, V, slice_bytes, on):
    """RECBLR_CE_GRADS=f16 (default): the logits' gradient in both layouts
    (rb_item_ce_probs_h_both) and both products on the f16 weight-gradient
    kernel (rb_gemm_tn_h) at the bench's shape (B = 2048, n_items = 10,544,
    d = 128) — no library GEMM runs — against torch fp64; shapes outside its
    conditions (B % 256, both layouts within the slice budget) take the sliced
    library path, same tolerance."""
    from datamining_recblr_amd import kernels, scoring

    monkeypatch.setattr(scoring, "PROBS_SLICE_BYTES", slice_bytes)
    monkeypatch.setattr(scoring, "CE_GRADS", "f16")
    seq, W, tgt = _data(B, V, 128, cuda, seed=15, scale=0.5)
    s1 = seq.clone().requires_grad_()
    w1 = W.clone().requires_grad_()
    mm = []
    orig = torch.mm
    monkeypatch.setattr(torch, "mm", lambda *a, **k: mm.append(1) or orig(*a, **k))
    with kernels.kernel_timing() as t:
        (0.7 * scoring.item_cross_entropy(s1, w1, tgt)).backward()
    names = {r[0] for r in t.records}
    if on:
        assert "rb_item_ce_probs_h_both" in names and not mm, (names, len(mm))
    else:
        assert "rb_item_ce_probs_h_both" not in names and mm, (names, len(mm))
    s2 = seq.double().requires_grad_()
    w2 = W.double().requires_grad_()
    (0.7 * F.cross_entropy(s2 @ w2.t(), tgt)).backward()
    normwise(s1.grad, s2.grad, 2e-5, "dseq")
    normwise(w1.grad, w2.grad, 2e-5, "ditems")
