"""GPU tests of the gates projection with the BD-LRU in its epilogue
(rb_gate_gemm_fwd_h, csrc/gemm_half.hip GATE; RecBLR.py:196-206: gates(x),
the alpha / beta gates, parallel_scan and silu(z) * h) on packed sequences.

Against the two-launch path it replaces — rb_gemm_nt_h (rg) followed by
rb_gate_scan_fwd (y, carries) on the same inputs:
  * rg bit for bit (the same main loop and row split);
  * y / y_last and the 16-step carries within fp32 re-association (the scan
    runs in 4-row groups, 32-row wave composites and 256-row tiles chained
    through the tails instead of 16-step chunks);
the whole model with the epilogue path engaged (asserted) against the CPU
oracle is tests/test_gpu_e2e.py (packed batches take it by default)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _packed(lens, L, dev):
    from datamining_recblr_amd import kernels

    B = len(lens)
    lens = torch.tensor(lens, dtype=torch.int64)
    order = torch.argsort(lens, descending=True, stable=True)
    offs = torch.zeros(B + 1, dtype=torch.int64)
    torch.cumsum(lens[order], 0, out=offs[1:])
    ntok = int(offs[-1])
    item_seq = torch.ones(B, L, dtype=torch.int64)
    ids, pos, inv, last, rinfo = kernels.pack_plan(item_seq.to(dev), offs.to(dev), order.to(dev),
                                                   ntok, want_rinfo=True)
    seq = kernels.Packed(offs.to(dev), L, ntok, pos)
    seq.last, seq.inv, seq.order, seq.rinfo = last, inv, order.to(dev), rinfo
    return seq


def _inputs(seq, H, dev, seed, tiny_rows=()):
    g = torch.Generator().manual_seed(seed)
    xz = torch.randn(seq.ntok, 2 * H, generator=g)
    xc = torch.nn.functional.silu(torch.randn(seq.ntok, H, generator=g))
    for r in tiny_rows:   # first 16 values far below the rest: the exact-recompute path
        xc[r, :16] *= 1e-30
    gw = torch.randn(2 * H, H, generator=g) / H ** 0.5
    gb = torch.randn(2 * H, generator=g) * 0.1
    lam = torch.linspace(-2.2, -6.9, H)
    h0 = torch.randn(H, generator=g)
    return (xz.to(dev), xc.to(dev), gw.to(dev), gb.to(dev), lam.to(dev), h0.to(dev))


def _carries_close(seq, c, c_r):
    """The carry slots of each sequence's own 16-step tiles (the rest of the
    [B, nT, H] buffer is never written nor read)."""
    lens = (seq.offsets[1:] - seq.offsets[:-1]).cpu()
    nt = (lens + 15) // 16
    valid = torch.arange(c.shape[1])[None, :] < nt[:, None]
    a, b = c.cpu()[valid], c_r.cpu()[valid]
    return _rel(a, b)


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


def _reference(seq, xz, xc, gw, gb, lam, h0, last_only, batch_row):
    from datamining_recblr_amd import kernels

    H = xc.shape[1]
    rg = kernels.gemm_nt_h(xc, kernels.gemm_h_weight(gw), 2 * H)
    y, carries = kernels.gate_scan_fwd(rg, xc, xz[:, H:], lam, h0, gate_b=gb, seq=seq,
                                       last_only=last_only, batch_row=batch_row)
    return rg, y, carries


def _fused(seq, xz, xc, gw, gb, lam, h0, last_only, batch_row):
    from datamining_recblr_amd import kernels

    H = xc.shape[1]
    return kernels.gate_gemm_fwd(xc, kernels.gemm_h_weight(gw), xz[:, H:], gb, lam, h0, seq,
                                 last_only=last_only, batch_row=batch_row)


def _lens(kind, g):
    if kind == "bench":      # RecBole-like ~U{1..200}, enough rows for the main phase
        return torch.randint(1, 201, (400,), generator=g).tolist()
    if kind == "ones":
        return [1] * 700
    if kind == "full256":    # whole tiles of one sequence each
        return [256] * 70 + [255, 1]
    if kind == "mixed":
        return [200, 1, 57, 256, 3, 129, 128, 17, 255, 2] * 25
    if kind == "small":      # below one round: the 256 x 64 phase only
        return torch.randint(1, 120, (37,), generator=g).tolist()
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["bench", "ones", "full256", "mixed", "small"])
@pytest.mark.parametrize("H", [256, 128])
@pytest.mark.parametrize("with_h0", [True, False])
def test_gate_gemm_equals_two_launch_path(cuda, kind, H, with_h0):
    from datamining_recblr_amd import kernels

    kinds = ["bench", "ones", "full256", "mixed", "small"]
    g = torch.Generator().manual_seed(10 * kinds.index(kind) + H)
    lens = _lens(kind, g)
    L = max(lens)
    seq = _packed(lens, L, cuda)
    xz, xc, gw, gb, lam, h0 = _inputs(seq, H, cuda, seed=len(lens) + H)
    h0 = h0 if with_h0 else None
    rg_r, y_r, c_r = _reference(seq, xz, xc, gw, gb, lam, h0, False, None)
    rg, y, c = _fused(seq, xz, xc, gw, gb, lam, h0, False, None)
    torch.cuda.synchronize()
    assert kernels.gate_gemm_errors() == 0
    assert torch.equal(rg, rg_r)
    assert _rel(y, y_r) < 2e-6, _rel(y, y_r)
    assert _carries_close(seq, c, c_r) < 2e-6, _carries_close(seq, c, c_r)


@pytest.mark.parametrize("kind", ["bench", "mixed"])
def test_gate_gemm_last_rows_in_batch_order(cuda, kind):
    """y only at each sequence's last row, written to its batch row (the last
    layer under gather_indexes, rb_gate_scan_fwd_last's contract)."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(5)
    lens = _lens(kind, g)
    seq = _packed(lens, max(lens), cuda)
    H = 256
    xz, xc, gw, gb, lam, h0 = _inputs(seq, H, cuda, seed=11)
    _, yl_r, c_r = _reference(seq, xz, xc, gw, gb, lam, h0, True, seq.order)
    _, yl, c = _fused(seq, xz, xc, gw, gb, lam, h0, True, seq.order)
    torch.cuda.synchronize()
    assert kernels.gate_gemm_errors() == 0
    assert _rel(yl, yl_r) < 2e-6 and _carries_close(seq, c, c_r) < 2e-6


def test_gate_gemm_flagged_rows(cuda):
    """Rows whose first 16 values are ~1e-30 of the rest overflow the online
    row scale: their tile is recomputed at exact scales inside the epilogue
    (the successor tile waits for it) — rg still bitwise the plain GEMM's."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(9)
    lens = _lens("bench", g)
    seq = _packed(lens, max(lens), cuda)
    H = 256
    tiny = [0, 255, 256, 5000, seq.ntok - 1]
    xz, xc, gw, gb, lam, h0 = _inputs(seq, H, cuda, seed=3, tiny_rows=tiny)
    rg_r, y_r, c_r = _reference(seq, xz, xc, gw, gb, lam, h0, False, None)
    rg, y, c = _fused(seq, xz, xc, gw, gb, lam, h0, False, None)
    torch.cuda.synchronize()
    assert kernels.gate_gemm_errors() == 0
    assert torch.equal(rg, rg_r)
    assert _rel(y, y_r) < 2e-6 and _carries_close(seq, c, c_r) < 2e-6


def test_gate_gemm_repeated_calls_and_rmax(cuda):
    """Back-to-back calls on one tails buffer (the epoch tags each call's
    tails), and the xc row-group maxima the weight-gradient kernel reads
    equal rb_gemm_nt_h's."""
    from datamining_recblr_amd import kernels

    g = torch.Generator().manual_seed(2)
    lens = _lens("bench", g)
    seq = _packed(lens, max(lens), cuda)
    H = 256
    xz, xc, gw, gb, lam, h0 = _inputs(seq, H, cuda, seed=4)
    img = kernels.gemm_h_weight(gw)
    rm_r = torch.empty((seq.ntok + 31) // 32, device=cuda)
    kernels.gemm_nt_h(xc, img, 2 * H, rmax=rm_r)
    outs = []
    for i in range(3):
        rm = torch.full_like(rm_r, -1.0)
        outs.append(kernels.gate_gemm_fwd(xc, img, xz[:, H:], gb, lam, h0, seq, rmax=rm))
        torch.cuda.synchronize()
        assert torch.equal(rm, rm_r)
    assert kernels.gate_gemm_errors() == 0
    for o in outs[1:]:   # deterministic: rg, y and the carry slots bit for bit
        assert torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1])
        assert _carries_close(seq, o[2], outs[0][2]) == 0.0
