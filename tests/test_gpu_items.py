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


@pytest.mark.parametrize("B,V,d", SHAPES)
def test_item_ce_matches_torch(cuda, B, V, d):
    from datamining_recblr_amd.scoring import item_cross_entropy

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
