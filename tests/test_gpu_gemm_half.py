"""GPU tests of the f16 two-part split fp32 GEMM (csrc/gemm_half.hip,
rb_gemm_nt_h) — the default projection GEMM (RECBLR_GEMM=f16x3) of F.linear's
forward and input-gradient products (RecBLR.py:162,165,167,213,214).

Every operand is scaled by an exact power of two and split into two fp16
parts; the error against an fp64 product is held to the level of torch's own
fp32 GEMM (hipBLASLt) on the same data, also on rows whose magnitudes span
the whole fp32 range (the per-row scale, and the exact recompute of rows that
outgrow their first scale)."""
import pytest
import torch
from tests.placement import bit31_alloc_bytes, bit31_offset

pytestmark = pytest.mark.gpu


def _rel_err(y, ref):
    return ((y.double() - ref).abs().max() / ref.abs().max()).item()


@pytest.mark.parametrize("M,K,N", [(4096, 128, 512), (5000, 256, 512), (4097, 512, 128),
                                   (8192, 256, 128), (300, 128, 256), (1, 32, 128),
                                   (257, 512, 384), (70001, 256, 512), (33, 1024, 1024)])
@pytest.mark.parametrize("bias", [False, True])
def test_forward_matches_fp64_at_fp32_accuracy(cuda, M, K, N, bias):
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(M + K + N)
    x = torch.randn(M, K, generator=g).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = torch.randn(N, generator=g).to(cuda) if bias else None
    y = kernels.gemm_nt_h(x, kernels.gemm_h_weight(w), N, bias=b)
    ref = x.double() @ w.double().t()
    if bias:
        ref = ref + b.double()
    yt = torch.addmm(b, x, w.t()) if bias else x @ w.t()
    e_h, e_torch = _rel_err(y, ref), _rel_err(yt, ref)
    # fp32-level: a few ulps of the output scale, on a par with hipBLASLt
    assert e_h < 2e-6, e_h
    assert e_h < 4 * max(e_torch, 1e-7), (e_h, e_torch)


@pytest.mark.parametrize("M,N,K", [(4096, 512, 128), (4100, 256, 512), (1024, 128, 256)])
def test_input_gradient_orientation(cuda, M, N, K):
    """Bm = W^T (the dX GEMM): the transposed image equals the image of the
    materialised transpose, bit for bit."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(7 * M + N)
    dy = torch.randn(M, N, generator=g).to(cuda)
    w = (torch.randn(N, K, generator=g) / N ** 0.5).to(cuda)
    wt = kernels.gemm_h_weight(w, transpose=True)
    assert torch.equal(wt.view(torch.int16),
                       kernels.gemm_h_weight(w.t().contiguous()).view(torch.int16))
    dx = kernels.gemm_nt_h(dy, wt, K)
    assert _rel_err(dx, dy.double() @ w.double()) < 2e-6


@pytest.mark.parametrize("N", [128, 512])
def test_rows_across_the_fp32_range(cuda, N):
    """Per-row relative error at fp32 level on rows scaled by 2^-60 .. 2^60,
    zero rows, rows whose first 16 (or 48) entries are zero or tiny and rows
    growing by 2^64 along K (their fp16 images would overflow the first
    scale: the kernel flags the tile and recomputes the wave's rows with the
    exact row max), a 3e37 entry; weight columns scaled by 1e-25 and zero.
    N = 128: 256 x 128 tiles with the deferred epilogue; N = 512: 256 x 256
    tiles stored at the tile's end."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(11)
    M, K = 4096 + 77, 256
    a = torch.randn(M, K, generator=g)
    a *= torch.exp2(torch.randint(-60, 60, (M, 1), generator=g).float())
    a[5] = 0
    a[6, :48] = 0
    a[7, :16] *= 1e-12
    a[8] *= torch.exp2(torch.arange(K).float() / 4)
    a[9, 100] = 3e37
    a[10] = 0
    a[10, 255] = 1e-30
    a[11, :200] = 1e-20
    a[300:340, :16] = 0          # a whole wave's rows flagged
    a = a.to(cuda)
    w = torch.randn(N, K, generator=g)
    w[3] *= 1e-25
    w[4, :10] = 0
    w[5] = 0
    w = w.to(cuda)
    ref = a.double() @ w.double().t()
    y = kernels.gemm_nt_h(a, kernels.gemm_h_weight(w), N)
    yt = a @ w.t()
    den = a.double().abs() @ w.double().abs().t()
    ok = den > 1e-30              # products inside fp32's normal range
    e_h = ((y.double() - ref).abs() / den)[ok].max().item()
    e_t = ((yt.double() - ref).abs() / den)[ok].max().item()
    assert torch.isfinite(y).all()
    assert e_h < 4 * max(e_t, 6e-8), (e_h, e_t)
    assert (y[5] == 0).all()


@pytest.mark.parametrize("N", [128, 512])
def test_non_finite_rows(cuda, N):
    """An inf or NaN entry of A: the outputs an fp32 GEMM makes non-finite
    are non-finite here too (NaN where torch gives ±inf: the split's low part
    of an infinite value is inf - inf), and every other row is unaffected —
    at fp32 accuracy, as without the bad rows."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(13)
    M, K = 4096 + 77, 256
    a = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    bad = [3, 300, 301, 4100]
    a_bad = a.clone()
    a_bad[3, 7] = float("inf")
    a_bad[300, 0] = -float("inf")
    a_bad[301, 200] = float("nan")
    a_bad[4100, 255] = float("inf")
    wi = kernels.gemm_h_weight(w.to(cuda))
    y = kernels.gemm_nt_h(a_bad.to(cuda), wi, N)
    yt = a_bad.to(cuda) @ w.to(cuda).t()
    assert torch.equal(torch.isfinite(y), torch.isfinite(yt))
    good = torch.ones(M, dtype=torch.bool)
    good[bad] = False
    assert not torch.isfinite(y[bad]).any()
    ref = (a.double() @ w.double().t())[good].to(cuda)
    assert _rel_err(y[good.to(cuda)], ref) < 2e-6


@pytest.mark.parametrize("mode", [0, 1], ids=["persistent", "weight_stationary"])
@pytest.mark.parametrize("M", [5000, 70001, 196608 + 8024])
@pytest.mark.parametrize("p,bias", [(0.0, True), (0.2, True), (0.2, False)])
def test_fused_activation_epilogue(cuda, M, p, bias, mode):
    """rb_gemm_nt_h_act (the FeedForward's w_1 with dropout(silu(.)) in the
    epilogue, RecBLR.py:219-221): out bit-identical to rb_gemm_nt_h with the
    bias, act bit-identical to rb_silu_dropout_fwd(out) with the same seed —
    on the persistent 256 x 256 launch, the 256 x 64 launch of the rows past
    the last whole round (Philox element index offset) and below one round;
    rows 7-9 and a wave's rows with zero prefixes force the cold recompute
    tail; the rmax side output equals the unfused GEMM's."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(M + int(10 * p))
    R, C = 128, 512
    a = torch.randn(M, R, generator=g)
    a[7, :16] = 0
    a[8, :16] *= 1e-12
    a[9] *= torch.exp2(torch.arange(R).float() / 4)
    a[300:340, :16] = 0
    a = a.to(cuda)
    w = (torch.randn(C, R, generator=g) / R ** 0.5).to(cuda)
    b = (0.1 * torch.randn(C, generator=g)).to(cuda) if bias else None
    wi = kernels.gemm_h_weight(w)
    nr = (M + 31) // 32
    r1 = torch.full((nr,), -1.0, device=cuda)
    r2 = torch.full((nr,), -1.0, device=cuda)
    with kernels.nt_h_mode(mode):   # (from 16,384 rows: mode 1 = gemm_ws.hip, EPI 1)
        out, act = kernels.gemm_nt_h_act(a, wi, C, b, seed=1234567, p=p, rmax=r1)
        ref = kernels.gemm_nt_h(a, wi, C, bias=b, rmax=r2)
    assert torch.equal(out, ref)
    assert torch.equal(act, kernels.silu_dropout_fwd(ref, seed=1234567, p=p))
    assert torch.equal(r1, r2)


@pytest.mark.parametrize("mode", [0, 1], ids=["persistent", "weight_stationary"])
@pytest.mark.parametrize("M", [5000, 70001, 196608 + 8024])
@pytest.mark.parametrize("p", [0.0, 0.2])
def test_fused_activation_backward_epilogue(cuda, M, p, mode):
    """rb_gemm_nt_h_dact (dU = dA2 W_2 with the activation's backward in the
    epilogue; dU never stored): da bit-identical to rb_gemm_nt_h +
    rb_silu_dropout_bwd with the same seed, on both launches (the 256 x 64 one
    with the Philox element offset) and below one round; rows 7-9 and a
    wave's rows with zero prefixes go through the cold recompute tail (their
    column sums from the recomputed values); dbias within fp32
    re-association of the unfused column partials, and deterministic; rmax
    as the unfused GEMM's."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(M + 3 + int(10 * p))
    R, C = 128, 512
    a = torch.randn(M, R, generator=g)
    a[7, :16] = 0
    a[8, :16] *= 1e-12
    a[9] *= torch.exp2(torch.arange(R).float() / 4)
    a[300:340, :16] = 0
    a = a.to(cuda)
    w = (torch.randn(R, C, generator=g) / R ** 0.5).to(cuda)   # mm_nn's w [N=R, K=C]
    pre = torch.randn(M, C, generator=g).to(cuda)
    wi = kernels.gemm_h_weight(w, transpose=True)
    nr = (M + 31) // 32
    r1 = torch.full((nr,), -1.0, device=cuda)
    r2 = torch.full((nr,), -1.0, device=cuda)
    with kernels.nt_h_mode(mode):   # (from 16,384 rows: mode 1 = gemm_ws.hip, EPI 2)
        da, db = kernels.gemm_nt_h_dact(a, wi, C, pre, seed=7654321, p=p, rmax=r1)
        du = kernels.gemm_nt_h(a, wi, C, rmax=r2)
        da2, db2 = kernels.gemm_nt_h_dact(a, wi, C, pre, seed=7654321, p=p)
    da_ref, db_ref = kernels.silu_dropout_bwd(pre, du, seed=7654321, p=p, want_dbias=True)
    assert torch.equal(da, da_ref)
    assert torch.equal(r1, r2)
    ref64 = da_ref.double().sum(0)
    tol = 1e-6 * da_ref.double().abs().sum(0).max().item()
    assert (db.double() - ref64).abs().max().item() < tol
    assert (db_ref.double() - ref64).abs().max().item() < tol
    assert torch.equal(da2, da) and torch.equal(db2, db)


def test_fused_activation_rejects_other_shapes(cuda):
    """The fused launch takes only shapes whose rows all run on a wide-epilogue
    launch (C % 256 == 0, not the few-rows kernel's shapes)."""
    from datamining_recblr_amd import kernels

    a = torch.randn(5000, 128, device=cuda)
    assert not kernels.gemm_nt_h_act_ok(a, 128)
    assert not kernels.gemm_nt_h_act_ok(a[:2048, :], 128)
    assert kernels.gemm_nt_h_act_ok(a, 512)
    with pytest.raises(ValueError):
        kernels.gemm_nt_h_act(a, kernels.gemm_h_weight(torch.randn(128, 128, device=cuda)), 128,
                              None, seed=1, p=0.1)


def test_row_strided_operand_and_output(cuda):
    """A as a column slice of a wider activation (the x half of xz), out as a
    row-strided view — the layouts the encoder hands over."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(3)
    big = torch.randn(4096, 512, generator=g).to(cuda)
    x = big[:, 256:]
    w = (torch.randn(256, 256, generator=g) / 16).to(cuda)
    outbig = torch.zeros(4096, 384, device=cuda)
    out = outbig[:, :256]
    kernels.gemm_nt_h(x, kernels.gemm_h_weight(w), 256, out=out)
    assert _rel_err(out, x.double() @ w.double().t()) < 2e-6
    assert outbig[:, 256:].abs().max().item() == 0.0


def test_row_group_max_side_output(cuda):
    """rmax[g] = max |A| over rows 32g .. 32g+31 (all columns), for a partial
    last group too — the weight-gradient kernel's operand scale."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(5)
    for M in (4096, 5000, 70001):
        a = (torch.randn(M, 256, generator=g) * torch.rand(M, 1, generator=g) * 100).to(cuda)
        w = torch.randn(512, 256, generator=g).to(cuda)
        rmax = torch.full(((M + 31) // 32,), -1.0, device=cuda)
        kernels.gemm_nt_h(a, kernels.gemm_h_weight(w), 512, rmax=rmax)
        ref = torch.nn.functional.pad(a.abs().amax(1), (0, (-M) % 32)).view(-1, 32).amax(1)
        assert torch.equal(rmax, ref)


def test_deterministic(cuda):
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(9)
    x = torch.randn(20000, 256, generator=g).to(cuda)
    wf = kernels.gemm_h_weight(torch.randn(512, 256, generator=g).to(cuda))
    y0 = kernels.gemm_nt_h(x, wf, 512)
    for _ in range(3):
        assert torch.equal(kernels.gemm_nt_h(x, wf, 512), y0)


def test_batched_weight_images_equal_single(cuda):
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


def test_layer_norm_backward_second_gradient(cuda):
    """rb_add_ln_bwd2: LN backward of dy + dy2 (added on load) equals the LN
    backward of the materialised sum, bit for bit."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(2)
    rows, d = 5000, 128
    a = torch.randn(rows, d, generator=g).to(cuda)
    r = torch.randn(rows, d, generator=g).to(cuda)
    gamma = torch.randn(d, generator=g).to(cuda)
    beta = torch.randn(d, generator=g).to(cuda)
    y, s, mean, rstd = kernels.add_ln_fwd(a, r, gamma, beta, 1e-12, save=True)
    dy = torch.randn(rows, d, generator=g).to(cuda)
    dy2 = torch.randn(rows, d, generator=g).to(cuda)
    one = kernels.add_ln_bwd(dy, s, gamma, mean, rstd, dy2=dy2, want_dbias=True)
    ref = kernels.add_ln_bwd(dy + dy2, s, gamma, mean, rstd, want_dbias=True)
    for x, xr in zip(one, ref):
        assert torch.equal(x, xr)


def _row_group_max(a):
    M = a.shape[0]
    return torch.nn.functional.pad(a.abs().amax(1), (0, (-M) % 32)).view(-1, 32).amax(1)


@pytest.mark.parametrize("M,N,K,S", [(204632, 512, 256, 64), (70001, 512, 128, 128),
                                     (4096 + 77, 128, 256, 256), (5000, 128, 512, 8),
                                     (300, 256, 128, 64), (2048 + 45, 10752, 128, 6),
                                     (3000, 128, 128, 5)])
def test_weight_gradient_tn_matches_fp64(cuda, M, N, K, S):
    """rb_gemm_tn_h: dW = dY^T X from fixed-order row-chunk partials (empty
    chunks write zeros) at fp32-level error next to hipBLASLt's fp32 GEMM, with
    the operand scales taken from the forward/input-gradient GEMMs' rmax."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(M + N + K)
    dy = (torch.randn(M, N, generator=g) * torch.rand(M, 1, generator=g) * 1e-3).to(cuda)
    x = (torch.randn(M, K, generator=g) * 3).to(cuda)
    ymax = torch.empty((M + 31) // 32, device=cuda)
    xmax = torch.empty((M + 31) // 32, device=cuda)
    # the side outputs of the GEMMs that read the same operands
    kernels.gemm_nt_h(dy, kernels.gemm_h_weight(torch.randn(128, N, device=cuda)), 128, rmax=ymax)
    kernels.gemm_nt_h(x, kernels.gemm_h_weight(torch.randn(128, K, device=cuda)), 128, rmax=xmax)
    assert torch.equal(ymax, _row_group_max(dy)) and torch.equal(xmax, _row_group_max(x))
    parts = kernels.gemm_tn_h(dy, x, ymax, xmax, S)
    assert parts.shape == (S, N, K)
    dw = kernels.colsum(parts.view(S, -1)).view(N, K)
    ref = dy.double().t() @ x.double()
    e_h = _rel_err(dw, ref)
    e_t = _rel_err(dy.t() @ x, ref)
    assert e_h < 2e-6 and e_h < 4 * max(e_t, 1e-7), (e_h, e_t)
    # deterministic
    assert torch.equal(kernels.gemm_tn_h(dy, x, ymax, xmax, S), parts)


@pytest.mark.parametrize("M,N,K", [(2048, 128, 512), (2048, 512, 128), (2048, 128, 256),
                                   (2500, 512, 256)])
def test_few_thousand_rows_weight_gradient_on_tn_kernel(cuda, monkeypatch, M, N, K):
    """linear.wgrad at the gathered last-layer tail's row counts (B = 2,048
    sequences): with both operands' rmax from the f16 GEMMs that read them
    (here the few-rows / 256 x 64-tile launches of rb_gemm_nt_h), the weight
    gradient runs on rb_gemm_tn_h with one 32-row group per split, at the
    same fp32-level error next to hipBLASLt."""
    from datamining_recblr_amd import kernels, linear

    monkeypatch.setattr(linear, "_tn_few", True)   # RECBLR_TN_FEW (default on)
    calls = []
    orig = kernels.gemm_tn_h
    monkeypatch.setattr(kernels, "gemm_tn_h", lambda *a, **k: calls.append(a[4]) or orig(*a, **k))
    g = torch.Generator().manual_seed(M + N + K)
    dy = (torch.randn(M, N, generator=g) * torch.rand(M, 1, generator=g) * 1e-3).to(cuda)
    x = (torch.randn(M, K, generator=g) * 3).to(cuda)
    ymax = torch.empty((M + 31) // 32, device=cuda)
    xmax = torch.empty((M + 31) // 32, device=cuda)
    kernels.gemm_nt_h(dy, kernels.gemm_h_weight(torch.randn(128, N, device=cuda)), 128, rmax=ymax)
    kernels.gemm_nt_h(x, kernels.gemm_h_weight(torch.randn(256, K, device=cuda)), 256, rmax=xmax)
    assert torch.equal(ymax, _row_group_max(dy)) and torch.equal(xmax, _row_group_max(x))
    dw = linear.wgrad(dy, x, ymax=ymax, xmax=xmax)
    assert len(calls) == 1 and calls[0] * 32 <= M, calls
    ref = dy.double().t() @ x.double()
    e_h = _rel_err(dw, ref)
    e_t = _rel_err(dy.t() @ x, ref)
    assert e_h < 2e-6 and e_h < 4 * max(e_t, 1e-7), (e_h, e_t)
    assert torch.equal(linear.wgrad(dy, x, ymax=ymax, xmax=xmax), dw)


def test_weight_gradient_rows_decaying_over_2_to_the_60(cuda):
    """Rows whose magnitudes decay by 2^60 along the chunk (the BD-LRU's
    alpha^t gradients): the per-chunk scale keeps the dominant rows exact and
    the tiny rows' contributions below fp32 rounding of the sum."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(4)
    M, N, K = 65536, 256, 128
    decay = torch.exp2(-(torch.arange(M) % 1000).float() * 0.06)[:, None]
    dy = (torch.randn(M, N, generator=g) * decay).to(cuda)
    x = torch.randn(M, K, generator=g).to(cuda)
    S = 64
    dw = kernels.colsum(kernels.gemm_tn_h(dy, x, _row_group_max(dy), _row_group_max(x), S)
                        .view(S, -1)).view(N, K)
    ref = dy.double().t() @ x.double()
    assert _rel_err(dw, ref) < 4 * max(_rel_err(dy.t() @ x, ref), 1e-7)


def test_weight_gradient_columns_spread_over_2_to_the_16(cuda):
    """Column magnitudes of dY and X spread over 2^16 (the TN kernel keeps
    one scale per operand and row chunk, shared by all columns: values within
    2^17 of the chunk max keep all 22 bits).  Checked per
    element at its own scale — dW[n, k] divided by the column scales
    cy[n] cx[k], so the small columns cannot hide behind the large ones — at
    the level of hipBLASLt's fp32 GEMM."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(9)
    M, N, K, S = 40000, 256, 128, 64
    cy = torch.exp2(-16.0 * torch.arange(N) / (N - 1))
    cx = torch.exp2(-16.0 * torch.arange(K) / (K - 1))
    dy = (torch.randn(M, N, generator=g) * cy).to(cuda)
    x = (torch.randn(M, K, generator=g) * cx).to(cuda)
    dw = kernels.colsum(kernels.gemm_tn_h(dy, x, _row_group_max(dy), _row_group_max(x), S)
                        .view(S, -1)).view(N, K)
    ref = dy.double().t() @ x.double()

    scale = (cy[:, None] * cx[None, :]).double().to(cuda)

    def scaled(out):
        return ((out.double() - ref).abs() / scale).max().item() / (ref.abs() / scale).max().item()

    e_h, e_t = scaled(dw), scaled(dy.t() @ x)
    assert e_h < 1e-5 and e_h < 4 * max(e_t, 1e-7), (e_h, e_t)


@pytest.mark.parametrize("spread", [24, 40])
@pytest.mark.parametrize("N,K", [(256, 128), (512, 256), (128, 512)])
def test_weight_gradient_columns_spread_beyond_2_to_the_16(cuda, spread, N, K):
    """Column magnitudes of dY and X spread over 2^24 and 2^40 inside every
    row chunk: the columns far below the chunk max would lose bits under the
    chunk's one scale, so the kernel detects them (the loaded values' column
    maxima) and redoes that tile's chunk with one exact power-of-two scale
    per column.  Per element at its own scale (dW[n, k] / (cy[n] cx[k])), at
    the level of hipBLASLt's fp32 GEMM; rows with ordinary magnitudes (no
    spread) take the one-pass path and stay bitwise as before."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(spread + N + K)
    M, S = 40000, 64
    cy = torch.exp2(-float(spread) * torch.arange(N) / (N - 1))
    cx = torch.exp2(-float(spread) * torch.arange(K) / (K - 1))
    dy = (torch.randn(M, N, generator=g) * cy).to(cuda)
    x = (torch.randn(M, K, generator=g) * cx).to(cuda)
    dw = kernels.colsum(kernels.gemm_tn_h(dy, x, _row_group_max(dy), _row_group_max(x), S)
                        .view(S, -1)).view(N, K)
    ref = dy.double().t() @ x.double()
    scale = (cy[:, None] * cx[None, :]).double().to(cuda)

    def scaled(out):
        return ((out.double() - ref).abs() / scale).max().item() / (ref.abs() / scale).max().item()

    e_h, e_t = scaled(dw), scaled(dy.t() @ x)
    assert e_h < 1e-5 and e_h < 4 * max(e_t, 1e-7), (e_h, e_t)


@pytest.mark.parametrize("M,K,N", [(2048, 512, 128), (2048, 128, 512), (2048, 256, 128),
                                   (77, 64, 32), (5000, 96, 96), (196608 + 8024, 256, 512),
                                   (196608 + 8024, 512, 128), (65536 * 3 + 31, 128, 256)])
def test_few_rows_kernel_and_round_remainder(cuda, M, K, N):
    """The few-rows kernel (csrc/gemm_small.hip: the gathered last-layer tail,
    B = 2048 rows; C % 128 != 0) and the rows past the persistent kernel's
    last whole round (bench-sized M: 196,608 rows there + 8,024 here, on the
    256 x 64-tile launch of the same kernel).  Every
    row at fp32 level against fp64 (per-row error against the row's max), the
    rmax side output equal to the exact 32-row-group maxima across the seam."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(M + 3 * K + N)
    x = (torch.randn(M, K, generator=g) * torch.exp2(torch.randint(-30, 30, (M, 1), generator=g)
                                                      .float())).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    rmax = torch.empty((M + 31) // 32, device=cuda)
    wf = kernels.gemm_h_weight(w)
    y = kernels.gemm_nt_h(x, wf, N, rmax=rmax)
    ref = x.double() @ w.double().t()
    row_err = ((y.double() - ref).abs().amax(1) / ref.abs().amax(1)).max().item()
    assert row_err < 4e-6, row_err
    # the bias epilogue: exactly the un-biased output plus the bias, in fp32
    assert torch.equal(kernels.gemm_nt_h(x, wf, N, bias=b), y + b)
    want = torch.nn.functional.pad(x.abs().amax(1), (0, (-M) % 32)).view(-1, 32).amax(1)
    assert torch.equal(rmax, want)


@pytest.mark.parametrize("M", [1, 100, 2048, 16383])
@pytest.mark.parametrize("N,K", [(128, 512), (512, 128), (128, 256), (64, 32)])
def test_few_rows_weight_gradient(cuda, M, N, K):
    """rb_gemm_tn_hs (the gathered tail's weight gradients, every M below
    linear.MIN_ROWS_FOR_SPLIT): per-column scales over each eighth of the
    rows, so columns spread over 2^±30 keep fp32-level accuracy per element
    at their own scale; accumulate adds into an existing dW."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(M + N + 7 * K)
    cy = torch.exp2(torch.randint(-30, 30, (N,), generator=g).float())
    cx = torch.exp2(torch.randint(-30, 30, (K,), generator=g).float())
    dy = (torch.randn(M, N, generator=g) * cy).to(cuda)
    x = (torch.randn(M, K, generator=g) * cx).to(cuda)
    dw = kernels.gemm_tn_hs(dy, x)
    ref = dy.double().t() @ x.double()
    scale = (cy[:, None] * cx[None, :]).double().to(cuda)
    err = ((dw.double() - ref).abs() / scale).max().item() / max(
        (ref.abs() / scale).max().item(), 1e-300)
    assert err < 4e-6, err
    base = torch.randn(N, K, generator=g).to(cuda)
    acc = base.clone()
    kernels.gemm_tn_hs(dy, x, out=acc, accumulate=True)
    assert torch.equal(acc, base + dw)
    assert torch.equal(kernels.gemm_tn_hs(dy, x), dw)   # deterministic


def _bit31_views(cuda, shapes):
    """fp32 views, 16-B aligned, whose device addresses all have bit 31 set
    (tests/placement.py), sliced from one allocation."""
    need = sum(4 * (r * c) + 256 for r, c in shapes)
    buf = torch.empty(bit31_alloc_bytes(need), dtype=torch.uint8, device=cuda)
    off = bit31_offset(buf.data_ptr(), need)
    views = []
    for r, c in shapes:
        v = buf[off: off + 4 * r * c].view(torch.float32).view(r, c)
        assert (v.data_ptr() >> 31) & 1 and v.data_ptr() % 16 == 0
        views.append(v)
        off += 4 * r * c + ((-(4 * r * c)) % 256)
    assert off <= buf.numel()
    return buf, views


@pytest.mark.parametrize("M,N,K,S", [(204632, 512, 256, 64), (5000, 128, 512, 8)])
def test_weight_gradient_tn_operands_above_bit_31(cuda, M, N, K, S):
    """rb_gemm_tn_h with both operands and the partials at addresses with
    bit 31 set, against fp64 and bitwise against the same operands placed by
    the allocator."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(31 + M)
    dy0 = (torch.randn(M, N, generator=g) * 1e-3).to(cuda)
    x0 = torch.randn(M, K, generator=g).to(cuda)
    buf, (dy, x) = _bit31_views(cuda, [(M, N), (M, K)])
    dy.copy_(dy0)
    x.copy_(x0)
    ymax, xmax = _row_group_max(dy0), _row_group_max(x0)
    parts = kernels.gemm_tn_h(dy, x, ymax, xmax, S)
    dw = kernels.colsum(parts.view(S, -1)).view(N, K)
    ref = dy0.double().t() @ x0.double()
    e_h = _rel_err(dw, ref)
    assert e_h < 2e-6 and e_h < 4 * max(_rel_err(dy0.t() @ x0, ref), 1e-7), e_h
    assert torch.equal(parts, kernels.gemm_tn_h(dy0, x0, ymax, xmax, S))
    del buf



@pytest.mark.parametrize("C,R", [(512, 128), (128, 512), (256, 48), (96, 16)])
def test_weight_image_strided_views_and_column_exponents(cuda, C, R):
    """rb_gemm_h_split_weights reads W along its rows (float4 runs when W is
    16-B aligned with ldw % 4 == 0, scalar loads otherwise): a row-strided
    view (ldw = R + 1) and a misaligned one give the image of the contiguous
    copy bit for bit, and the column exponents are frexp of each column's
    max |Bm| (both orientations)."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(C + R)
    base = (torch.randn(C, R + 1, generator=g) *
            torch.exp2(torch.randint(-30, 30, (C, 1), generator=g).float())).to(cuda)
    wv = base[:, :R]                 # ldw = R + 1
    wm = base[:, 1:]                 # ldw = R + 1, 4-B offset: not 16-B aligned
    for w in (wv, wm):
        ref = kernels.gemm_h_weight(w.contiguous())
        assert torch.equal(kernels.gemm_h_weight(w).view(torch.int16), ref.view(torch.int16))
        e = ref.view(torch.int32)[C * R:C * R + C]
        m = w.abs().amax(1)
        assert torch.equal(e.cpu(), torch.frexp(m.cpu())[1].to(torch.int32))
    bt = torch.randn(R, C + 1, generator=g).to(cuda)[:, :C]   # W [R, C], ldw = C + 1
    wt = kernels.gemm_h_weight(bt, transpose=True)             # Bm = W^T
    assert torch.equal(wt.view(torch.int16),
                       kernels.gemm_h_weight(bt.t().contiguous()).view(torch.int16))


# ---- the weight-stationary kernel (csrc/gemm_ws.hip; rb_gemm_nt_h from 16,384 rows)

WS_SHAPES = [(128, 512), (512, 128), (256, 512), (512, 256), (256, 128), (128, 256)]


def _adversarial_rows(a):
    """rows over 2^+-60, zero rows, zero / tiny prefixes (the persistent
    kernel's recompute tail), growth by 2^32 along K, a 3e30 entry"""
    M, K = a.shape
    g = torch.Generator().manual_seed(M + K)
    a *= torch.exp2(torch.randint(-60, 60, (M, 1), generator=g).float())
    a[5] = 0
    a[6, :K // 4] = 0
    a[7, :16] *= 1e-12
    a[8] = torch.randn(K, generator=g) * torch.exp2(torch.arange(K).float() * (32.0 / K))
    a[9] = torch.randn(K, generator=g)
    a[9, K // 2] = 3e30
    a[31] = 0
    a[32] = 0
    a[32, K - 1] = 1e-30
    a[M - 1] = torch.randn(K, generator=g) * 2.0 ** 40
    return a


@pytest.mark.parametrize("R,C", WS_SHAPES)
@pytest.mark.parametrize("M", [16384, 16384 + 32 * 257 + 5, 204632])
def test_ws_kernel_matches_fp64_per_row(cuda, R, C, M):
    """The encoder's projection shapes on the weight-stationary kernel: every
    output element of 600 sampled rows (the block edges, the partial last
    block, adversarial rows) within fp32 accuracy of fp64 relative to
    sum |a||b| (the dot product's own rounding scale), on a par with
    hipBLASLt's fp32 GEMM on the same rows; bias; rmax exact; rows past M
    untouched; the persistent kernel (mode 0) agrees at the same bar."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(M + R + C)
    a = _adversarial_rows(torch.randn(M, R, generator=g))
    w = torch.randn(C, R, generator=g) / R ** 0.5
    w[3] *= 1e-25
    w[5] = 0
    b = torch.randn(C, generator=g)
    a, w, b = a.to(cuda), w.to(cuda), b.to(cuda)
    wi = kernels.gemm_h_weight(w)
    outbig = torch.full((M + 3, C), 7.0, device=cuda)
    out = outbig[:M]
    nr = (M + 31) // 32
    rmax = torch.full((nr,), -1.0, device=cuda)
    assert kernels.gemm_nt_h_mode() == 1
    kernels.gemm_nt_h(a, wi, C, bias=b, out=out, rmax=rmax)
    assert (outbig[M:] == 7.0).all()
    ref_rmax = torch.nn.functional.pad(a.abs().amax(1), (0, (-M) % 32)).view(-1, 32).amax(1)
    assert torch.equal(rmax, ref_rmax)
    rows = torch.cat([torch.arange(0, 40), torch.arange(M - 40, M),
                      torch.randint(0, M, (520,), generator=g)]).unique()
    ad, wd = a[rows].double().cpu(), w.double().cpu()
    ref = ad @ wd.t() + b.double().cpu()
    den = ad.abs() @ wd.abs().t() + b.double().cpu().abs()
    ok = den > 1e-30
    y = out[rows].double().cpu()
    yt = (a[rows] @ w.t() + b).double().cpu()
    e_h = ((y - ref).abs() / den)[ok].max().item()
    e_t = ((yt - ref).abs() / den)[ok].max().item()
    assert torch.isfinite(out).all()
    assert e_h < 4 * max(e_t, 6e-8), (e_h, e_t)
    with kernels.nt_h_mode(0):
        y0 = kernels.gemm_nt_h(a, wi, C, bias=b)[rows].double().cpu()
    assert (((y0 - ref).abs() / den)[ok].max().item()) < 4 * max(e_t, 6e-8)


def test_ws_kernel_non_finite_rows_and_transpose(cuda):
    """inf / NaN entries poison exactly their rows (as the fp32 GEMM's,
    NaN where it gives +-inf); the transposed weight image (the dX GEMM's
    Bm = W^T) gives the same outputs as the image of the materialised
    transpose; bitwise deterministic; differs from the persistent kernel only
    at rounding level (so the two kernels are distinct launches)."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(17)
    M, N, K = 40000 + 13, 512, 256       # dY [M, N] @ W [N, K]
    dy = torch.randn(M, N, generator=g)
    bad = [3, 33, 20000, M - 1]
    dy[3, 7] = float("inf")
    dy[33, 0] = -float("inf")
    dy[20000, 300] = float("nan")
    dy[M - 1, 511] = float("inf")
    dy = dy.to(cuda)
    w = (torch.randn(N, K, generator=g) / N ** 0.5).to(cuda)
    wt = kernels.gemm_h_weight(w, transpose=True)
    dx = kernels.gemm_nt_h(dy, wt, K)
    bits = lambda t: t.view(torch.int32)   # noqa: E731 (NaN rows compare by bits)
    assert torch.equal(bits(dx), bits(kernels.gemm_nt_h(dy, kernels.gemm_h_weight(w.t().contiguous()), K)))
    assert torch.equal(bits(dx), bits(kernels.gemm_nt_h(dy, wt, K)))
    ref = dy @ w
    assert torch.equal(torch.isfinite(dx), torch.isfinite(ref))
    good = torch.ones(M, dtype=torch.bool, device=cuda)
    good[bad] = False
    assert not torch.isfinite(dx[~good]).any()
    r64 = dy[good].double() @ w.double()
    assert _rel_err(dx[good], r64) < 2e-6
    with kernels.nt_h_mode(0):
        dx0 = kernels.gemm_nt_h(dy, wt, K)
    assert not torch.equal(dx0[good], dx[good])
    assert _rel_err(dx0[good], r64) < 2e-6


def test_ws_kernel_row_strided_views(cuda):
    """A as the z half of an [M, 2H] activation (row stride 2H), out a
    column slice of a wider buffer (the dxz halves the encoder hands over)."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(23)
    M = 30000
    big = torch.randn(M, 512, generator=g).to(cuda)
    x = big[:, 256:]
    w = (torch.randn(256, 256, generator=g) / 16).to(cuda)
    outbig = torch.zeros(M, 512, device=cuda)
    out = outbig[:, 256:]
    kernels.gemm_nt_h(x, kernels.gemm_h_weight(w), 256, out=out)
    assert _rel_err(out, x.double() @ w.double().t()) < 2e-6
    assert outbig[:, :256].abs().max().item() == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("K", [128, 256, 512])
@pytest.mark.parametrize("M", [16384 + 37, 70000])
@pytest.mark.parametrize("p,bias", [(0.0, False), (0.2, True)])
def test_ln_epilogue_matches_gemm_then_add_ln(cuda, K, M, p, bias):
    """rb_gemm_nt_h_ln (the weight-stationary kernel's LayerNorm epilogue,
    RecBLR.py:142, 225-227) == rb_gemm_nt_h + rb_add_ln_fwd: s bit for bit
    (the same GEMM output and Philox keep-flags), mean / rstd / y within fp32
    re-association of the row moments; and against fp64 LayerNorm of s."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(31 + K)
    d = 128
    a = torch.randn(M, K, generator=g).to(cuda)
    w = (torch.randn(d, K, generator=g) / K ** 0.5).to(cuda)
    b = (0.1 * torch.randn(d, generator=g)).to(cuda) if bias else None
    r = torch.randn(M, d, generator=g)
    r[::97] += 300.0                                  # rows whose mean dwarfs their spread
    r = r.to(cuda)
    gamma = (1 + 0.1 * torch.randn(d, generator=g)).to(cuda)
    beta = (0.1 * torch.randn(d, generator=g)).to(cuda)
    wi = kernels.gemm_h_weight(w)
    rm = torch.empty((M + 31) // 32, device=cuda)
    with kernels.nt_h_mode(1):
        assert kernels.gemm_nt_h_ln_ok(a, d)
        y, s, mean, rstd = kernels.gemm_nt_h_ln(a, wi, d, b, r, gamma, beta, 1e-12, 77, p, rmax=rm)
        o = kernels.gemm_nt_h(a, wi, d, bias=b)
    y2, s2, mean2, rstd2 = kernels.add_ln_fwd(o, r, gamma, beta, 1e-12, seed=77, p=p)
    assert torch.equal(s, s2)
    assert torch.equal(rm, _row_group_max(a))
    sd = s2.double()
    md = sd.mean(1)
    vd = ((sd - md[:, None]) ** 2).mean(1)
    yd = (sd - md[:, None]) / torch.sqrt(vd[:, None] + 1e-12) * gamma.double() + beta.double()
    scale = sd.abs().amax(1)
    assert ((mean.double() - md).abs() / scale).max().item() < 1e-6
    assert ((rstd.double() - 1 / torch.sqrt(vd + 1e-12)).abs() / rstd.double()).max().item() < 2e-5
    assert (y.double() - yd).abs().max().item() < 2e-4
    # the same rounding class as rb_add_ln_fwd's two-pass moments
    assert (y - y2).abs().max().item() < 2e-4
    assert ((rstd - rstd2).abs() / rstd2).max().item() < 2e-5


@pytest.mark.gpu
def test_ln_epilogue_needs_the_weight_stationary_kernel(cuda):
    """rb_gemm_nt_h_ln runs only on the weight-stationary kernel: with
    rb_gemm_nt_h_mode 0 the eligibility check says no and a direct call fails
    loudly (no silent fallback)."""
    from datamining_recblr_amd import _lib, kernels

    M, d = 20000, 128
    a = torch.randn(M, 256, device=cuda)
    w = torch.randn(d, 256, device=cuda) / 16
    r = torch.randn(M, d, device=cuda)
    one = torch.ones(d, device=cuda)
    with kernels.nt_h_mode(0):
        assert not kernels.gemm_nt_h_ln_ok(a, d)
        with pytest.raises(_lib.RecBLRNativeError):
            _lib.call("rb_gemm_nt_h_ln", a.data_ptr(), 256, M, 256,
                      kernels.gemm_h_weight(w).data_ptr(), d, 0, r.data_ptr(), one.data_ptr(),
                      one.data_ptr(), 1e-12, 0, 0.0, r.data_ptr(), r.data_ptr(), one.data_ptr(),
                      one.data_ptr(), d, 0, 0)
