"""GPU parity of the fused blocks around the BD-LRU against plain torch fp32
compositions of the reference's ops (RecBLR.py:76-78, :142, :210-227).  Both
sides drop the same elements: either an explicit mask is passed to the
kernels, or the kernels' Philox keep-mask is materialised (rb_dropout_mask)
and applied on the torch side."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def close(a, b, atol=1e-5, rtol=1e-5, what=""):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    err = (a - b).abs()
    bad = err > atol + rtol * b.abs() + 2e-6 * b.abs().max()
    assert not bad.any(), f"{what}: max err {err.max().item():.3e}"


def _mask(g, shape, p, cuda):
    return (torch.rand(shape, generator=g) >= p).to(torch.uint8).to(cuda) if p else None


@pytest.mark.parametrize("rows,d", [(7, 16), (33, 64), (1000, 128), (129, 256), (64, 512),
                                    (5, 1024), (409, 32)])
@pytest.mark.parametrize("mode", ["none", "mask", "philox"])
def test_add_dropout_layer_norm(cuda, rows, d, mode):
    from datamining_recblr_amd import kernels
    from datamining_recblr_amd.blocks import _AddDropoutLN

    p = 0.0 if mode == "none" else 0.2
    g = torch.Generator(device="cpu").manual_seed(rows * d)
    a = torch.randn(rows, d, generator=g).to(cuda).requires_grad_()
    r = torch.randn(rows, d, generator=g).to(cuda).requires_grad_()
    gamma = (1 + 0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_()
    beta = (0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_()
    dy = torch.randn(rows, d, generator=g).to(cuda)
    seed = 1234 + rows
    if mode == "mask":
        mask = _mask(g, (rows, d), p, cuda)
        ref_mask = mask
    else:
        mask = None
        ref_mask = kernels.dropout_mask(seed, p, (rows, d), cuda) if p else None
    y = _AddDropoutLN.apply(a, r, gamma, beta, mask, seed, p, 1e-12)
    y.backward(dy)
    ar, rr, gr, br = (t.detach().clone().requires_grad_() for t in (a, r, gamma, beta))
    dropped = ar * ref_mask / (1 - p) if ref_mask is not None else ar
    yr = F.layer_norm(dropped + rr, (d,), gr, br, eps=1e-12)
    yr.backward(dy)
    close(y, yr, what="y")
    close(a.grad, ar.grad, atol=1e-4, what="da")
    close(r.grad, rr.grad, atol=1e-4, what="dr")
    close(gamma.grad, gr.grad, atol=1e-4, rtol=1e-4, what="dgamma")
    close(beta.grad, br.grad, atol=1e-4, rtol=1e-4, what="dbeta")


def test_philox_mask_statistics_and_determinism(cuda):
    from datamining_recblr_amd import kernels

    m1 = kernels.dropout_mask(7, 0.2, (4096, 512), cuda)
    m2 = kernels.dropout_mask(7, 0.2, (4096, 512), cuda)
    m3 = kernels.dropout_mask(8, 0.2, (4096, 512), cuda)
    assert torch.equal(m1, m2) and not torch.equal(m1, m3)
    keep = m1.float().mean().item()
    assert abs(keep - 0.8) < 2e-3, keep
    # no structure along rows or columns: every row / column mean within 6
    # binomial standard deviations of 0.8
    sd_row, sd_col = (0.16 / 512) ** 0.5, (0.16 / 4096) ** 0.5
    assert (m1.float().mean(1) - 0.8).abs().max() < 6 * sd_row
    assert (m1.float().mean(0) - 0.8).abs().max() < 6 * sd_col
    # consecutive elements (one Philox call covers 4) are not correlated
    f = m1.float().view(-1)
    corr = ((f[:-1] - 0.8) * (f[1:] - 0.8)).mean().item() / 0.16
    assert abs(corr) < 0.01, corr


@pytest.mark.parametrize("p", [0.0, 0.2])
def test_embed_dropout_layer_norm(cuda, p):
    """Gather + dropout + LN, and the deterministic embedding backward, incl.
    padding id 0, a very popular id (multi-chunk segment sums) and unused ids."""
    from datamining_recblr_amd import kernels
    from datamining_recblr_amd.blocks import _EmbedDropoutLN

    V, d, B, L = 500, 128, 16, 300
    g = torch.Generator(device="cpu").manual_seed(11)
    table = torch.randn(V, d, generator=g).to(cuda).requires_grad_()
    idx = torch.randint(0, V // 2, (B, L), generator=g)
    idx[:, ::3] = 7          # 1600 occurrences of one id -> 25 chunks
    idx[:, -5:] = 0          # padding
    idx = idx.to(cuda)
    gamma = (1 + 0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_()
    beta = (0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_()
    dy = torch.randn(B, L, d, generator=g).to(cuda)
    seed = 99
    y = _EmbedDropoutLN.apply(table, idx, gamma, beta, None, seed, p, 1e-12, 0)
    y.backward(dy)
    tr, gr, br = (t.detach().clone().requires_grad_() for t in (table, gamma, beta))
    e = F.embedding(idx, tr, padding_idx=0)
    if p:
        e = e * kernels.dropout_mask(seed, p, (B, L, d), cuda) / (1 - p)
    yr = F.layer_norm(e, (d,), gr, br, eps=1e-12)
    yr.backward(dy)
    close(y, yr, what="y")
    close(table.grad, tr.grad, atol=1e-4, rtol=1e-4, what="dtable")
    assert table.grad[0].abs().max().item() == 0.0
    assert table.grad[V // 2:].abs().max().item() == 0.0
    close(gamma.grad, gr.grad, atol=1e-4, rtol=1e-4, what="dgamma")
    close(beta.grad, br.grad, atol=1e-4, rtol=1e-4, what="dbeta")


def test_embedding_bwd_skewed_and_deterministic(cuda):
    from datamining_recblr_amd import kernels

    V, d, M = 10544, 128, 409600
    g = torch.Generator(device="cpu").manual_seed(5)
    # Zipf-like: a few ids take most of the mass
    w = 1.0 / torch.arange(1, V + 1, dtype=torch.float64) ** 1.1
    idx = torch.multinomial(w, M, replacement=True, generator=g).to(cuda)
    grad = torch.randn(M, d, generator=g).to(cuda)
    dw = kernels.embedding_bwd(idx, grad, V, padding_idx=0)
    ref = torch.zeros(V, d, dtype=torch.float64, device=cuda).index_add_(0, idx, grad.double())
    ref[0] = 0
    close(dw, ref.float(), atol=1e-3, rtol=1e-5, what="dW")
    assert torch.equal(dw, kernels.embedding_bwd(idx, grad, V, padding_idx=0))


@pytest.mark.parametrize("M", [1, 63, 257, 16385, 409600])
def test_embedding_counting_sort_plan_equals_radix_plan(cuda, M):
    """Tables up to 16384 rows are planned by the four-launch counting sort,
    larger ones by the rocPRIM radix sort; both order each id's positions
    ascending, so the segment sums are bitwise equal (the larger table's
    extra rows stay zero).  Ragged M: fewer rows than row blocks, partial
    64-row steps."""
    from datamining_recblr_amd import kernels

    V, d = 10544, 64
    g = torch.Generator(device="cpu").manual_seed(M)
    w = 1.0 / torch.arange(1, V + 1, dtype=torch.float64) ** 1.1
    idx = torch.multinomial(w, M, replacement=True, generator=g).to(cuda)
    grad = torch.randn(M, d, generator=g).to(cuda)
    small = kernels.embedding_bwd(idx, grad, V, padding_idx=0)
    big = kernels.embedding_bwd(idx, grad, 16385, padding_idx=0)
    assert torch.equal(small, big[:V])
    assert big[V:].abs().max().item() == 0.0
    ref = torch.zeros(V, d, dtype=torch.float64, device=cuda).index_add_(0, idx, grad.double())
    ref[0] = 0
    close(small, ref.float(), atol=1e-3, rtol=1e-5, what="dW")


@pytest.mark.parametrize("mode", ["none", "mask", "philox"])
def test_silu_dropout(cuda, mode):
    from datamining_recblr_amd import kernels
    from datamining_recblr_amd.blocks import _SiluDropout

    p = 0.0 if mode == "none" else 0.3
    g = torch.Generator(device="cpu").manual_seed(3)
    a = (3 * torch.randn(37, 512, generator=g)).to(cuda).requires_grad_()
    du = torch.randn(37, 512, generator=g).to(cuda)
    seed = 5
    mask = _mask(g, (37, 512), p, cuda) if mode == "mask" else None
    ref_mask = mask if mode == "mask" else (kernels.dropout_mask(seed, p, (37, 512), cuda)
                                            if p else None)
    u = _SiluDropout.apply(a, mask, seed, p)
    u.backward(du)
    ar = a.detach().clone().requires_grad_()
    ur = F.silu(ar)
    if ref_mask is not None:
        ur = ur * ref_mask / (1 - p)
    ur.backward(du)
    close(u, ur, what="u")
    close(a.grad, ar.grad, what="da")


@pytest.mark.parametrize("p", [0.0, 0.2])
def test_fused_feed_forward(cuda, p, split_gemm_calls):
    """_FeedForward (two GEMMs, SiLU+dropout, dropout+residual+LN, folded bias
    grads, residual grad through addmm) == the reference FeedForward math.
    M = 5000 rows: all four fwd/dX GEMMs run the f16x3 kernel (asserted)."""
    from datamining_recblr_amd import kernels
    from datamining_recblr_amd.blocks import _FeedForward

    g = torch.Generator(device="cpu").manual_seed(21)
    M, d = 5000, 128
    x = torch.randn(M, d, generator=g).to(cuda).requires_grad_()
    w1 = (0.05 * torch.randn(4 * d, d, generator=g)).to(cuda).requires_grad_()
    b1 = (0.1 * torch.randn(4 * d, generator=g)).to(cuda).requires_grad_()
    w2 = (0.05 * torch.randn(d, 4 * d, generator=g)).to(cuda).requires_grad_()
    b2 = (0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_()
    gamma = (1 + 0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_()
    beta = (0.1 * torch.randn(d, generator=g)).to(cuda).requires_grad_()
    dy = torch.randn(M, d, generator=g).to(cuda)
    s1, s2 = 31, 32
    y = _FeedForward.apply(x, w1, b1, w2, b2, gamma, beta, s1, s2, p, 1e-12)
    y.backward(dy)
    assert sorted(split_gemm_calls) == sorted([(M, d, 4 * d), (M, 4 * d, d), (M, d, 4 * d),
                                               (M, 4 * d, d)]), split_gemm_calls
    leaves = [t.detach().clone().requires_grad_() for t in (x, w1, b1, w2, b2, gamma, beta)]
    xr, w1r, b1r, w2r, b2r, gr, br = leaves
    h = F.silu(F.linear(xr, w1r, b1r))
    if p:
        h = h * kernels.dropout_mask(s1, p, (M, 4 * d), cuda) / (1 - p)
    h = F.linear(h, w2r, b2r)
    if p:
        h = h * kernels.dropout_mask(s2, p, (M, d), cuda) / (1 - p)
    yr = F.layer_norm(h + xr, (d,), gr, br, eps=1e-12)
    yr.backward(dy)
    close(y, yr, atol=1e-4, what="y")
    for name, a, b in zip(("dx", "dw1", "db1", "dw2", "db2", "dgamma", "dbeta"),
                          (x, w1, b1, w2, b2, gamma, beta), leaves):
        close(a.grad, b.grad, atol=1e-4, rtol=1e-4, what=name)


@pytest.mark.parametrize("M", [20000, 204632])
def test_feed_forward_fused_activation_bitwise(cuda, M):
    """The FeedForward with w_1's activation in the forward GEMM's epilogue
    and its backward in the dU GEMM's (RECBLR_FFN_ACT, linear.mm_nt_act /
    mm_nn_dact) == the GEMMs + rb_silu_dropout_fwd/bwd path, bit for bit: the
    output and every gradient but db1 (the w_1 bias gradient: the same
    values summed in another fixed order, within fp32 re-association)."""
    from datamining_recblr_amd import kernels, linear
    from datamining_recblr_amd.blocks import _FeedForward

    g = torch.Generator(device="cpu").manual_seed(22)
    d = 128
    base = [torch.randn(M, d, generator=g), 0.05 * torch.randn(4 * d, d, generator=g),
            0.1 * torch.randn(4 * d, generator=g), 0.05 * torch.randn(d, 4 * d, generator=g),
            0.1 * torch.randn(d, generator=g), 1 + 0.1 * torch.randn(d, generator=g),
            0.1 * torch.randn(d, generator=g)]
    dy = torch.randn(M, d, generator=g).to(cuda)
    res = []
    # fused vs unfused, bitwise on either NT kernel (rb_gemm_nt_h_mode 0: the
    # persistent tiles; 1: the weight-stationary kernel, EPI 1 / 2, from
    # 16,384 rows); the two kernels agree at fp32 accuracy
    # (the LayerNorm epilogue off: its row moments are another fp32 order)
    for fused, mode in ((True, 0), (False, 0), (True, 1), (False, 1)):
        prev = linear.set_ffn_act_fused(fused)
        prev_ln = linear.set_ln_fused(False)
        try:
            with kernels.nt_h_mode(mode):
                leaves = [t.to(cuda).requires_grad_() for t in base]
                assert linear.mm_nt_act_ok(leaves[0], leaves[1]) == fused
                assert linear.mm_nn_dact_ok(dy, leaves[3]) == fused
                y = _FeedForward.apply(*leaves, 41, 42, 0.2, 1e-12)
                y.backward(dy)
                res.append([y.detach()] + [t.grad for t in leaves])
        finally:
            linear.set_ffn_act_fused(prev)
            linear.set_ln_fused(prev_ln)
    names = ("y", "dx", "dw1", "db1", "dw2", "db2", "dgamma", "dbeta")
    for f, u_ in ((0, 1), (2, 3)):
        for name, u, v in zip(names, res[f], res[u_]):
            if name == "db1":
                close(u, v, atol=1e-6 * v.abs().max().item(), rtol=1e-5, what=name)
            else:
                assert torch.equal(u, v), name
    for name, u, v in zip(names, res[3], res[1]):
        close(u, v, atol=1e-5 * v.abs().max().item(), rtol=1e-5, what=name + " (ws)")


@pytest.mark.parametrize("M", [20000, 204632])
def test_feed_forward_ln_epilogue(cuda, M, monkeypatch):
    """The FeedForward with the residual + dropout + LayerNorm in w_2's GEMM
    epilogue (RECBLR_LN_EPI, linear.mm_nt_ln: rb_add_ln_fwd gone) == the GEMM
    + rb_add_ln_fwd path: the output and every gradient within fp32 rounding
    of the row moments (the same s, the same keep-flags)."""
    from datamining_recblr_amd import kernels, linear
    from datamining_recblr_amd.blocks import _FeedForward

    g = torch.Generator(device="cpu").manual_seed(23)
    d = 128
    base = [torch.randn(M, d, generator=g), 0.05 * torch.randn(4 * d, d, generator=g),
            0.1 * torch.randn(4 * d, generator=g), 0.05 * torch.randn(d, 4 * d, generator=g),
            0.1 * torch.randn(d, generator=g), 1 + 0.1 * torch.randn(d, generator=g),
            0.1 * torch.randn(d, generator=g)]
    dy = torch.randn(M, d, generator=g).to(cuda)
    res = []
    for on in (True, False):
        prev = linear.set_ln_fused(on)
        calls = []
        orig = kernels.add_ln_fwd
        monkeypatch.setattr(kernels, "add_ln_fwd", lambda *a, **k: calls.append(1) or orig(*a, **k))
        try:
            with kernels.nt_h_mode(1):
                leaves = [t.to(cuda).requires_grad_() for t in base]
                u = torch.empty(M, 4 * d, device=cuda)
                assert linear.mm_nt_ln_ok(u, leaves[3]) == on
                y = _FeedForward.apply(*leaves, 51, 52, 0.2, 1e-12)
                y.backward(dy)
                res.append([y.detach()] + [t.grad for t in leaves])
        finally:
            linear.set_ln_fused(prev)
            monkeypatch.setattr(kernels, "add_ln_fwd", orig)
        assert len(calls) == (0 if on else 1)
    names = ("y", "dx", "dw1", "db1", "dw2", "db2", "dgamma", "dbeta")
    for name, u, v in zip(names, res[0], res[1]):
        close(u, v, atol=2e-5 * v.abs().max().item(), rtol=1e-4, what=name + " (ln epilogue)")


def test_recurrent_layer_out_projection_ln_epilogue(cuda, monkeypatch):
    """RecurrentLayer with the out-projection and its residual LayerNorm in
    one launch (RecBLR.py:142, 167: rb_gemm_nt_h_ln, rb_add_ln_fwd not called
    for that LayerNorm) == the projection + rb_add_ln_fwd path: output and
    every parameter / input gradient within fp32 rounding of the LayerNorm
    moments, in train mode with dropout (same seeds)."""
    from datamining_recblr_amd import blocks, kernels, linear
    from datamining_recblr_amd.model import RecurrentLayer

    torch.manual_seed(3)
    layer = RecurrentLayer(d_model=128, d_conv=4, expand=2, dropout=0.2, num_layers=2,
                           bd_lru_only=False, disable_conv1d=False, disable_ffn=False).to(cuda)
    layer.train()
    g = torch.Generator(device="cpu").manual_seed(4)
    x0 = torch.randn(96, 200, 128, generator=g).to(cuda)   # 19,200 rows
    dy = torch.randn(96, 200, 128, generator=g).to(cuda)
    res = []
    for on in (True, False):
        prev = linear.set_ln_fused(on)
        calls = []
        orig = kernels.gemm_nt_h_ln
        monkeypatch.setattr(kernels, "gemm_nt_h_ln", lambda *a, **k: calls.append(a[0].shape[1]) or orig(*a, **k))
        try:
            torch.manual_seed(11)   # the same dropout seeds both ways
            layer.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_()
            y = layer(x)
            y.backward(dy)
            res.append([y.detach(), x.grad] + [p.grad.clone() for p in layer.parameters()])
        finally:
            linear.set_ln_fused(prev)
            monkeypatch.setattr(kernels, "gemm_nt_h_ln", orig)
        # the out-projection (K = 256) and the FeedForward's w_2 (K = 512)
        assert sorted(calls) == ([256, 512] if on else []), calls
    names = ["y", "dx"] + [n for n, _ in layer.named_parameters()]
    for name, u, v in zip(names, res[0], res[1]):
        close(u, v, atol=2e-5 * v.abs().max().item(), rtol=1e-4, what=name + " (out-proj ln)")


def test_train_mode_dropout(cuda):
    """Train-mode model: fresh dropout per call (outputs differ run to run),
    reproducible under torch.manual_seed, and p = 0 in train mode == eval."""
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset

    cfg = dict(hidden_size=64, loss_type="CE", num_layers=2, dropout_prob=0.2, expand=2,
               d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
               MAX_ITEM_LIST_LENGTH=50)
    torch.manual_seed(0)
    model = RecBLR(cfg, SyntheticDataset(300)).to(cuda)
    seq = torch.randint(1, 300, (32, 50), device=cuda)
    lens = torch.randint(1, 51, (32,), device=cuda)
    model.train()
    torch.manual_seed(5)
    a = model.forward(seq, lens)
    b = model.forward(seq, lens)
    torch.manual_seed(5)
    a2 = model.forward(seq, lens)
    assert not torch.equal(a, b)
    assert torch.equal(a, a2)
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    c = model.forward(seq, lens)
    model.eval()
    close(c, model.forward(seq, lens), what="p=0 train == eval")


@pytest.mark.parametrize("M", [1000, 409600, 409637])
def test_split_k_weight_gradient(cuda, M):
    """linear.LinearFn: forward == F.linear, split-K dW (incl. a ragged tail) ==
    the plain GEMM within fp32 re-association error."""
    from datamining_recblr_amd.linear import LinearFn, wgrad

    g = torch.Generator(device="cpu").manual_seed(M)
    x = torch.randn(M, 128, generator=g).to(cuda).requires_grad_()
    w = (0.05 * torch.randn(256, 128, generator=g)).to(cuda).requires_grad_()
    b = torch.randn(256, generator=g).to(cuda).requires_grad_()
    dy = torch.randn(M, 256, generator=g).to(cuda)
    y = LinearFn.apply(x, w, b)
    y.backward(dy)
    xr, wr, br = (t.detach().clone().requires_grad_() for t in (x, w, b))
    F.linear(xr, wr, br).backward(dy)
    close(y, F.linear(xr, wr, br), atol=1e-4, what="y")
    close(x.grad, xr.grad, atol=1e-4, what="dx")
    ref = (dy.double().t() @ x.detach().double()).float()
    close(w.grad, ref, atol=1e-3, rtol=1e-5, what="dW")
    close(b.grad, br.grad, atol=1e-3, rtol=1e-5, what="db")
    assert torch.equal(wgrad(dy, x.detach()), wgrad(dy, x.detach()))


@pytest.mark.parametrize("H,pads", [(256, 56), (128, 14), (512, 1), (64, [0, 3, 14, 56, 1000]),
                                    (128, 0)])
def test_pad_prefix_kernels_match_torch(cuda, H, pads):
    """rb_pad_prefix_fwd/_bwd against the torch statement pad_prefix_state
    and its autograd (shared and per-row pad lengths)."""
    from datamining_recblr_amd.recurrence import PadPrefix, pad_prefix_state

    g = torch.Generator(device="cpu").manual_seed(H)
    cb = (0.5 * torch.randn(H, generator=g)).to(cuda)
    gw = (0.1 * torch.randn(2 * H, H, generator=g)).to(cuda)
    gb = (0.1 * torch.randn(2 * H, generator=g)).to(cuda)
    lam = torch.linspace(-2.0, 1.0, H).to(cuda)
    P = torch.tensor(pads, device=cuda) if isinstance(pads, list) else pads
    a = [t.clone().requires_grad_() for t in (cb, gw, gb, lam)]
    b = [t.clone().double().requires_grad_() for t in (cb, gw, gb, lam)]
    h_k = PadPrefix.apply(*a, P)
    h_t = pad_prefix_state(*b, P)
    close(h_k, h_t, atol=1e-5, rtol=1e-5, what="h0")
    dh = torch.randn(h_t.shape, generator=g).to(cuda)
    (h_k * dh).sum().backward()
    (h_t * dh.double()).sum().backward()
    for x, y, n in zip(a, b, ("dconv_b", "dgate_w", "dgate_b", "dlam")):
        err = (x.grad.double() - y.grad).norm() / max(y.grad.norm().item(), 1e-30)
        assert err < 2e-5, (n, err.item())


@pytest.mark.parametrize("shape", [(1, 1), (7, 3), (64, 131072), (128, 65536), (512, 16384),
                                   (1024, 128), (300, 65),
                                   (3, 2048, 256), (2048, 1024), (2048, 256), (2000, 256)])
def test_colsum_fixed_order(cuda, shape):
    from datamining_recblr_amd import kernels

    g = torch.Generator(device="cpu").manual_seed(sum(shape))
    x = torch.randn(shape, generator=g).to(cuda)
    out = kernels.colsum(x)
    ref = x.double().sum(-2)
    assert out.shape == ref.shape
    close(out, ref, atol=1e-5, rtol=1e-5, what="colsum")
    assert torch.equal(out, kernels.colsum(x))
    # restated order: RG interleaved partials in increasing p, combined in order
    # (RG = 4 for P <= 256, else 16; 16 for wide partials, C >= 8192 and
    # P >= 64); few columns with many rows: 64-row chunk sums first, then the
    # chunk sums (kernels.colsum)
    def one_pass(xs):
        P, C = xs.shape[1], xs.shape[2]
        RG = 16 if (C >= 8192 and P >= 64 and C % 4 == 0) else (4 if P <= 256 else 16)
        parts = [torch.zeros(xs.shape[0], xs.shape[2]) for _ in range(RG)]
        for p in range(P):
            parts[p % RG] = parts[p % RG] + xs[:, p]
        exp = parts[0]
        for q in parts[1:]:
            exp = exp + q
        return exp

    P, C = shape[-2], shape[-1]
    xs = x.reshape(-1, P, C).cpu()
    M = xs.shape[0]
    if M * ((C + 63) // 64) < 64 and P >= 256 and P % 64 == 0:
        exp = one_pass(one_pass(xs.reshape(M * (P // 64), 64, C)).reshape(M, P // 64, C))
    else:
        exp = one_pass(xs)
    assert torch.equal(out.cpu().reshape(exp.shape), exp)


def test_silu_dropout_with_folded_bias(cuda):
    from datamining_recblr_amd import kernels

    g = torch.Generator(device="cpu").manual_seed(4)
    a = torch.randn(65, 256, generator=g).to(cuda)
    b = torch.randn(256, generator=g).to(cuda)
    du = torch.randn(65, 256, generator=g).to(cuda)
    u = kernels.silu_dropout_fwd(a, seed=9, p=0.25, bias=b)
    keep = kernels.dropout_mask(9, 0.25, (65, 256), cuda).float() / 0.75
    close(u, F.silu(a + b) * keep, what="u")
    da, db = kernels.silu_dropout_bwd(a, du, seed=9, p=0.25, want_dbias=True, bias=b)
    ar = (a + b).requires_grad_()
    (F.silu(ar) * keep).backward(du)
    close(da, ar.grad, what="da")
    close(db, ar.grad.double().sum(0), what="db")


@pytest.mark.parametrize("H,K,dt", [(64, 4, torch.float32), (20, 3, torch.float32),
                                    (256, 4, torch.float32), (64, 8, torch.float32),
                                    (128, 4, torch.bfloat16), (64, 1, torch.float32)])
def test_conv_rows_equals_per_sequence(cuda, H, K, dt):
    """rb_conv_silu_fwd_rows (packed rows tiled directly, row positions mask
    the history) == rb_conv_silu_fwd on the same packed sequences (per-sequence
    tiles) bit for bit, lengths 1..40 incl. single-row sequences, on a
    row-strided view (the in-projection's x half)."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(H * 10 + K)
    lens = torch.randint(1, 41, (37,), generator=g)
    lens[3] = 1
    lens[5] = 40
    offs = torch.zeros(lens.numel() + 1, dtype=torch.int64)
    torch.cumsum(lens, 0, out=offs[1:])
    ntok = int(offs[-1])
    xz = torch.randn(ntok, 2 * H, generator=g).to(dt).to(cuda)
    w = (torch.randn(H, 1, K, generator=g) * 0.4).to(cuda)
    b = (torch.randn(H, generator=g) * 0.1).to(cuda)
    offs_d = offs.to(cuda)
    pos = (torch.arange(ntok) - offs[:-1].repeat_interleave(lens)).to(cuda)
    x = xz[:, :H]
    ref = kernels.conv_silu_fwd(x, w, b, kernels.Packed(offs_d, 40, ntok))
    out = kernels.conv_silu_fwd(x, w, b, kernels.Packed(offs_d, 40, ntok, pos))
    assert out.dtype == dt
    assert torch.equal(out, ref)
    # and against the definition: each sequence alone, zero history
    xf = x.float().cpu()
    for s in (0, 3, 5):
        a, e = int(offs[s]), int(offs[s + 1])
        xs = torch.nn.functional.pad(xf[a:e].t()[None], (K - 1, 0))
        y = torch.nn.functional.silu(torch.nn.functional.conv1d(xs, w.cpu(), b.cpu(), groups=H))
        tol = 1e-5 if dt == torch.float32 else 1e-2
        assert (out[a:e].float().cpu() - y[0].t()).abs().max().item() < tol


def test_gate_scan_last_only_equals_full(cuda):
    """rb_gate_scan_fwd_last / _bwd_last (only each packed sequence's last
    position of y kept; dy given there only) == the full kernels with y
    gathered at those rows and dy zero elsewhere, bit for bit."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(17)
    H = 64
    lens = torch.randint(1, 60, (23,), generator=g)
    lens[0], lens[4] = 1, 59
    lens = lens.sort(descending=True).values
    offs = torch.zeros(lens.numel() + 1, dtype=torch.int64)
    torch.cumsum(lens, 0, out=offs[1:])
    ntok, B = int(offs[-1]), lens.numel()
    rg = torch.randn(ntok, 2 * H, generator=g).to(cuda)
    xz = torch.randn(ntok, 2 * H, generator=g).to(cuda)
    xc, z = xz[:, :H], xz[:, H:]
    lam = torch.linspace(-2.2, -6.9, H).to(cuda)
    gb = (0.1 * torch.randn(2 * H, generator=g)).to(cuda)
    h0 = torch.randn(H, generator=g).to(cuda)
    seq = kernels.Packed(offs.to(cuda), 64, ntok)
    last = (offs[1:] - 1).to(cuda)
    y, car = kernels.gate_scan_fwd(rg, xc, z, lam, h0, gate_b=gb, seq=seq)
    yl, carl = kernels.gate_scan_fwd(rg, xc, z, lam, h0, gate_b=gb, seq=seq, last_only=True)
    assert torch.equal(yl, y.index_select(0, last))
    # carries [B, nT, H]: a packed sequence writes only its own ceil(len / 16)
    # tiles; the rest of the buffer is never written (torch.empty) nor read
    for s in range(B):
        nt = (int(lens[s]) + kernels.RB_TILE - 1) // kernels.RB_TILE
        assert torch.equal(carl[s, :nt], car[s, :nt]), s
    dyl = torch.randn(B, H, generator=g).to(cuda)
    dy = torch.zeros(ntok, H, device=cuda)
    dy.index_copy_(0, last, dyl)
    dz1, dz2 = torch.empty(ntok, H, device=cuda), torch.empty(ntok, H, device=cuda)
    r1 = kernels.gate_scan_bwd(rg, xc, z, lam, car, dy, dz1, gate_b=gb, seq=seq)
    r2 = kernels.gate_scan_bwd(rg, xc, z, lam, car, dyl, dz2, gate_b=gb, seq=seq, last_only=True)
    assert torch.equal(dz1, dz2)
    for a, b in zip(r1, r2):
        assert torch.equal(a, b)
    # batch_row: sequence s's row of y_last / dy_last is perm[s]
    perm = torch.randperm(B, generator=g).to(cuda)
    yp, _ = kernels.gate_scan_fwd(rg, xc, z, lam, h0, gate_b=gb, seq=seq, last_only=True,
                                  batch_row=perm)
    assert torch.equal(yp.index_select(0, perm), yl)
    dyp = torch.empty_like(dyl)
    dyp[perm] = dyl
    dz3 = torch.empty(ntok, H, device=cuda)
    r3 = kernels.gate_scan_bwd(rg, xc, z, lam, car, dyp, dz3, gate_b=gb, seq=seq, last_only=True,
                               batch_row=perm)
    assert torch.equal(dz1, dz3)
    for a, b in zip(r1, r3):
        assert torch.equal(a, b)


def test_last_only_model_equals_full_positions(cuda):
    """RecBLR's packed last layer with the last-position scan kernels gives the
    same loss and gradients, bit for bit, as keeping y at every position."""
    from datamining_recblr_amd import model as M
    from datamining_recblr_amd.distributed import synthetic_interaction
    from datamining_recblr_amd.recbole_compat import SyntheticDataset

    cfg = dict(hidden_size=64, loss_type="CE", num_layers=2, dropout_prob=0.0, expand=2,
               d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
               MAX_ITEM_LIST_LENGTH=50)
    inter = synthetic_interaction(128, 50, 300, cuda, seed=4)
    res = []
    for flag in (True, False):
        M._LAST_ONLY = flag
        torch.manual_seed(0)
        model = M.RecBLR(cfg, SyntheticDataset(300)).to(cuda).train()
        loss = model.calculate_loss(inter)
        loss.backward()
        res.append((loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters()
                                    if p.grad is not None}))
    M._LAST_ONLY = True
    assert torch.equal(res[0][0], res[1][0])
    for n in res[0][1]:
        assert torch.equal(res[0][1][n], res[1][1][n]), n


def test_pack_plan_matches_torch(cuda):
    """rb_pack_plan == the torch index/scatter formulation of the packed layout."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(8)
    B, L = 37, 70
    item_seq = torch.randint(1, 500, (B, L), generator=g)
    lens = torch.randint(1, L + 1, (B,), generator=g)
    lens[2], lens[5] = 1, L
    order = torch.argsort(lens, descending=True, stable=True)
    offs = torch.zeros(B + 1, dtype=torch.int64)
    torch.cumsum(lens[order], 0, out=offs[1:])
    ntok = int(offs[-1])
    ids, pos, inv, last = kernels.pack_plan(item_seq.to(cuda), offs.to(cuda), order.to(cuda), ntok)
    seq_of = torch.repeat_interleave(torch.arange(B), lens[order])
    pos_r = torch.arange(ntok) - offs[seq_of]
    ids_r = item_seq.reshape(-1)[order[seq_of] * L + pos_r]
    inv_r = torch.empty_like(order)
    inv_r[order] = torch.arange(B)
    assert torch.equal(ids.cpu(), ids_r) and torch.equal(pos.cpu(), pos_r)
    assert torch.equal(inv.cpu(), inv_r) and torch.equal(last.cpu(), offs[inv_r + 1] - 1)


@pytest.mark.parametrize("pads", [56, [0, 3, 14, 56]])
def test_folded_pad_prefix_equals_separate_node(cuda, pads):
    """bd_lru folds the pad-prefix state into BDLRUCore (its backward adds
    into the parameter gradients in place, rb_pad_prefix_bwd accumulate=1):
    bit-identical outputs and gradients to PadPrefix + BDLRUCore with an
    explicit h0, where autograd sums the two contributions."""
    from datamining_recblr_amd.recurrence import BDLRUCore, PadPrefix, bd_lru

    B, L, H, K = 4, 72, 128, 4
    g = torch.Generator(device="cpu").manual_seed(7)
    xz = torch.randn(B, L, 2 * H, generator=g).to(cuda)
    params = [(0.3 * torch.randn(H, 1, K, generator=g)).to(cuda),
              (0.5 * torch.randn(H, generator=g)).to(cuda),
              (0.1 * torch.randn(2 * H, H, generator=g)).to(cuda),
              (0.1 * torch.randn(2 * H, generator=g)).to(cuda),
              torch.linspace(-2.0, 1.0, H).to(cuda)]
    pad = torch.tensor(pads, device=cuda) if isinstance(pads, list) else None
    dy = torch.randn(B, L, H, generator=g).to(cuda)
    outs = []
    for fold in (True, False):
        x = xz.clone().requires_grad_()
        p = [t.clone().requires_grad_() for t in params]
        if fold:
            y = bd_lru(x, *p, use_conv=True, pad=pad)
        else:
            h0 = PadPrefix.apply(*p[1:], pad if pad is not None else pads)
            y = BDLRUCore.apply(x, *p, h0, True, None, False)
        (y * dy).sum().backward()
        outs.append([y.detach(), x.grad] + [t.grad for t in p])
    for a, b, n in zip(*outs, ("y", "dxz", "dconv_w", "dconv_b", "dgate_w", "dgate_b", "dlam")):
        assert torch.equal(a, b), n


@pytest.mark.parametrize("K,dt", [(4, torch.float32), (3, torch.float32), (4, torch.bfloat16)])
def test_conv_bwd_folded_partials_equal_separate(cuda, K, dt):
    """rb_conv_silu_bwd with db_part NULL (folded per-sequence partials:
    [dW in [c, k] order | dbias] per row, one column sum) writes bit for bit
    the values of the separate dw_part[b, k, c] / db_part[b, c] layout, and
    the same dx."""
    from datamining_recblr_amd import _lib
    from datamining_recblr_amd.kernels import _stream

    g = torch.Generator().manual_seed(K)
    B, L, H = 9, 37, 64
    sfx = "_bf16" if dt == torch.bfloat16 else ""
    xz = torch.randn(B, L, 2 * H, generator=g).to(dt).to(cuda)
    x = xz[..., :H]
    w = (torch.randn(H, K, generator=g) * 0.4).to(cuda)
    b = (torch.randn(H, generator=g) * 0.1).to(cuda)
    g1 = torch.randn(B, L, H, generator=g).to(dt).to(cuda)
    g2 = torch.randn(B, L, H, generator=g).to(dt).to(cuda)
    outs = []
    for folded in (False, True):
        dx = torch.empty(B, L, 2 * H, dtype=dt, device=cuda)[..., :H]
        if folded:
            part = torch.full((B, (K + 1) * H), float("nan"), device=cuda)
            ptrs = (part.data_ptr(), 0)
        else:
            dwp = torch.full((B, K, H), float("nan"), device=cuda)
            dbp = torch.full((B, H), float("nan"), device=cuda)
            ptrs = (dwp.data_ptr(), dbp.data_ptr())
        _lib.call("rb_conv_silu_bwd" + sfx, x.data_ptr(), 2 * H, w.data_ptr(), b.data_ptr(),
                  g1.data_ptr(), g2.data_ptr(), dx.data_ptr(), 2 * H, *ptrs, B, L, H, K, None,
                  _stream(x))
        torch.cuda.synchronize()
        if folded:
            outs.append((dx.clone(), part[:, :H * K].view(B, H, K), part[:, H * K:]))
        else:
            outs.append((dx.clone(), dwp.permute(0, 2, 1), dbp))
    (dx0, dw0, db0), (dx1, dw1, db1) = outs
    assert torch.equal(dx0, dx1)
    assert torch.equal(dw0, dw1)
    assert torch.equal(db0, db1)


def test_gate_bwd_pattern_probe_covers_every_element(cuda):
    """rb_probe_gate_bwd_pattern (bench.py's pattern ceiling) touches exactly
    the gate backward's elements: on a packed batch (lengths 1..37, paired
    longest-first waves) every output row of every sequence is written with
    its trivial product, and nothing past ntok."""
    from datamining_recblr_amd import _lib
    from datamining_recblr_amd.kernels import _stream

    g = torch.Generator().manual_seed(3)
    H = 64
    lens = torch.randint(1, 38, (23,), generator=g).sort(descending=True).values
    offs = torch.zeros(lens.numel() + 1, dtype=torch.int64)
    torch.cumsum(lens, 0, out=offs[1:])
    ntok = int(offs[-1])
    rg = torch.randn(ntok, 2 * H, generator=g).to(cuda)
    xz = torch.randn(ntok, 2 * H, generator=g).to(cuda)
    xc = torch.randn(ntok, H, generator=g).to(cuda)
    dy = torch.randn(ntok, H, generator=g).to(cuda)
    drg = torch.full((ntok + 5, 2 * H), float("nan"), device=cuda)
    dxc = torch.full((ntok + 5, H), float("nan"), device=cuda)
    dxz = torch.full((ntok + 5, 2 * H), float("nan"), device=cuda)
    z, dz = xz[:, H:], dxz[:, H:]
    _lib.call_probe("rb_probe_gate_bwd_pattern", rg.data_ptr(), 2 * H, xc.data_ptr(), H, z.data_ptr(),
              2 * H, dy.data_ptr(), drg.data_ptr(), 2 * H, dxc.data_ptr(), H, dz.data_ptr(), 2 * H,
              lens.numel(), 37, H, offs.to(cuda).data_ptr(), _stream(xc))
    torch.cuda.synchronize()
    assert torch.equal(drg[:ntok, :H], rg[:, :H] * dy)
    assert torch.equal(drg[:ntok, H:], rg[:, H:] * dy)
    assert torch.equal(dxc[:ntok], xc * dy)
    assert torch.equal(dz[:ntok], z * dy)
    assert torch.isnan(drg[ntok:]).all() and torch.isnan(dxc[ntok:]).all()
    assert torch.isnan(dxz[:, :H]).all() and torch.isnan(dxz[ntok:]).all()


@pytest.mark.parametrize("M,R,C", [(1, 128, 512), (37, 512, 128), (1000, 256, 256)])
def test_gemm_pattern_probe_covers_every_output(cuda, M, R, C):
    """rb_probe_gemm_pattern (bench.py gemm.pattern) reads every A row and
    writes every output of the GEMM it stands in for (out[m, 4j + i] =
    rowsum(a[m]) + i), nothing past M rows."""
    from datamining_recblr_amd import _lib
    from datamining_recblr_amd.kernels import _stream

    g = torch.Generator().manual_seed(M + R)
    a = torch.randn(M, R, generator=g).to(cuda)
    out = torch.full((M + 3, C), float("nan"), device=cuda)
    _lib.call_probe("rb_probe_gemm_pattern", a.data_ptr(), M, R, out.data_ptr(), C, _stream(a))
    torch.cuda.synchronize()
    ref = a.double().sum(1, keepdim=True) + (torch.arange(C, device=cuda) % 4).double()[None]
    assert torch.allclose(out[:M].double(), ref, atol=1e-3, rtol=1e-5)
    assert torch.isnan(out[M:]).all()


@pytest.mark.parametrize("shape", [(3, 2048, 256), (2048, 256), (1024, 512), (4096, 128)])
def test_colsum_chunked_one_launch_equals_two_passes(cuda, shape):
    """rb_colsum_chunked (chunk sums, then the last arriving workgroup of each
    column block sums them) is bitwise the two rb_colsum passes it replaced,
    call after call: the tickets reset themselves and the workspace's lines,
    reused by the allocator, are re-read after the acquire."""
    from datamining_recblr_amd import _lib, kernels
    from datamining_recblr_amd.kernels import _stream

    g = torch.Generator(device=cuda).manual_seed(sum(shape))
    P, C = shape[-2], shape[-1]
    M = 1 if len(shape) == 2 else shape[0]
    nch = P // 64
    for it in range(60):
        x = torch.randn(shape, device=cuda, generator=g) * (1 + it % 7)
        out = kernels.colsum(x)
        part = torch.empty(M * nch, C, device=cuda)
        ref = torch.empty(M, C, device=cuda)
        _lib.call("rb_colsum", x.data_ptr(), M * nch, 64, C, C, 64 * C, part.data_ptr(), _stream(x))
        _lib.call("rb_colsum", part.data_ptr(), M, nch, C, C, nch * C, ref.data_ptr(), _stream(x))
        assert torch.equal(out.reshape(M, C), ref), it
    tickets = kernels._tickets[(x.device, _stream(x))]
    assert int(tickets.abs().sum()) == 0



def test_colsum_chunked_tickets_dropped_after_a_failed_call(cuda):
    """The tickets stay in [0, nch) (the kernel's wrapping increment) and are
    back at 0 after every complete launch; a failed native call drops the
    cached counters altogether (_lib.on_failure), so the next call starts
    from fresh zeros and is exact."""
    from datamining_recblr_amd import _lib, kernels
    from datamining_recblr_amd.kernels import _stream

    x = torch.randn(2048, 256, device=cuda)
    ref = kernels.colsum(x).clone()
    key = (x.device, _stream(x))
    assert int(kernels._tickets[key].abs().sum()) == 0
    with pytest.raises(_lib.RecBLRNativeError):
        _lib.call("rb_colsum", 0, 1, 1, 1, 1, 1, 0, 0)
    assert key not in kernels._tickets
    assert torch.equal(kernels.colsum(x), ref)
    assert int(kernels._tickets[key].abs().sum()) == 0
