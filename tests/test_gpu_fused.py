"""The fused GatedRecurrentLayer forward and backward (experimental/grl_fused.hip,
rb_grl_fwd / rb_grl_bwd): conv + SiLU, the behaviour-gate projection and the
BD-LRU scan with the silu(z) merge in one launch each way (RecBLR.py:182-206),
against the three-launch path they replace (rb_conv_silu_fwd_rows,
rb_gemm_nt_h, rb_gate_scan_fwd and the mirror-image backward) on the same
packed batch, and the whole model with them against the unfused model.

Bars: xc bit-identical (the same conv arithmetic); rg within fp32 level of
the row's magnitude (both are f16x3 GEMMs; the scales differ); y, the
16-step carries and y_last within 1e-5 relative to the tensor's max (the scan
composes its 4-row groups in a different order); xc's 32-row-group maxima
exact."""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.experimental]


def _packed_batch(cuda, B, L, H, seed, fixed=False):
    from datamining_recblr_amd import kernels
    from datamining_recblr_amd.kernels import Packed, grl_pieces

    g = torch.Generator().manual_seed(seed)
    lens = torch.full((B,), L) if fixed else torch.randint(1, L + 1, (B,), generator=g)
    lens_p = lens.sort(descending=True).values
    offs = torch.zeros(B + 1, dtype=torch.int64)
    torch.cumsum(lens_p, 0, out=offs[1:])
    ntok = int(offs[-1])
    pos = torch.cat([torch.arange(n) for n in lens_p.tolist()])
    seq = Packed(offs.to(cuda), L, ntok, pos.to(cuda))
    G = torch.cuda.get_device_properties(cuda).multi_processor_count
    seq.pieces, seq.G = grl_pieces(lens_p, offs, G).to(cuda), G
    seq.max_tiles = kernels.grl_max_tiles(lens_p, G)
    xz = torch.randn(ntok, 2 * H, generator=g).to(cuda)
    conv_w = (torch.randn(H, 1, 4, generator=g) * 0.5).to(cuda)
    conv_b = (torch.randn(H, generator=g) * 0.1).to(cuda)
    gate_w = (torch.randn(2 * H, H, generator=g) / H ** 0.5).to(cuda)
    gate_b = (torch.randn(2 * H, generator=g) * 0.1).to(cuda)
    lam = torch.linspace(-2.1972, -6.9068, H).to(cuda)
    h0 = (torch.randn(H, generator=g) * 0.3).to(cuda)
    return kernels, seq, xz, conv_w, conv_b, gate_w, gate_b, lam, h0


def _rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("B,L,fixed", [(2048, 200, False), (192, 200, True), (300, 50, False),
                                       (7, 3, False), (64, 1, False), (1000, 130, False)])
def test_fused_forward_matches_three_launch_path(cuda, B, L, fixed):
    kernels, seq, xz, conv_w, conv_b, gate_w, gate_b, lam, h0 = _packed_batch(cuda, B, L, 256,
                                                                            B + L, fixed)
    H = 256
    x, z = xz[:, :H], xz[:, H:]
    # reference: the three launches
    xc_ref = kernels.conv_silu_fwd(x, conv_w, conv_b, seq=seq)
    wf = kernels.gemm_h_weight(gate_w)
    rg_ref = kernels.gemm_nt_h(xc_ref, wf, 2 * H)
    y_ref, car_ref = kernels.gate_scan_fwd(rg_ref, xc_ref, z, lam, h0, gate_b=gate_b, seq=seq)
    ylast_ref, _ = kernels.gate_scan_fwd(rg_ref, xc_ref, z, lam, h0, gate_b=gate_b, seq=seq,
                                         last_only=True, want_carries=False)
    y, car, xc, rg, rmax = kernels.grl_fwd(xz, conv_w, conv_b, wf, gate_b, lam, h0, seq)
    torch.cuda.synchronize()
    assert torch.equal(xc, xc_ref)
    row_err = ((rg - rg_ref).abs().amax(1) / rg_ref.abs().amax(1).clamp_min(1e-30)).max().item()
    assert row_err < 4e-6, row_err
    assert _rel(y, y_ref) < 1e-5
    # carries: only the checkpoints the sequences reach are defined
    nT = car.shape[1]
    lens = (seq.offsets[1:] - seq.offsets[:-1]).cpu()
    mask = (torch.arange(nT)[None, :] * 16 < lens[:, None]).to(cuda)
    assert _rel(car[mask], car_ref[mask]) < 1e-5
    want = torch.nn.functional.pad(xc_ref.abs().amax(1), (0, (-xc.shape[0]) % 32)).view(-1, 32)
    assert torch.equal(rmax, want.amax(1))
    ylast, *_ = kernels.grl_fwd(xz, conv_w, conv_b, wf, gate_b, lam, h0, seq, want_y=False,
                                want_train=False)
    assert _rel(ylast, ylast_ref) < 1e-5
    # deterministic
    y2, *_ = kernels.grl_fwd(xz, conv_w, conv_b, wf, gate_b, lam, h0, seq)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("last_only", [False, True], ids=["all_rows", "last_rows"])
@pytest.mark.parametrize("B,L,fixed", [(2048, 200, False), (192, 200, True), (300, 50, False),
                                       (7, 3, False), (64, 1, False), (1000, 130, False)])
def test_fused_backward_matches_three_launch_path(cuda, B, L, fixed, last_only):
    """rb_grl_bwd (from rb_grl_fwd's 64-row tile checkpoints) against
    rb_gate_scan_bwd + the dxc GEMM + rb_conv_silu_bwd on the same batch:
    xc bit-identical; dz, dx, drg and the parameter gradients within 1e-5 of
    the tensor's max (the gates GEMM's f16x3 scales differ per row / tile;
    the partial sums group differently); the 32-row maxima exact."""
    kernels, seq, xz, conv_w, conv_b, gate_w, gate_b, lam, h0 = _packed_batch(cuda, B, L, 256,
                                                                            7 * B + L, fixed)
    H = 256
    x, z = xz[:, :H], xz[:, H:]
    g = torch.Generator().manual_seed(B)
    dy = torch.randn((seq.B if last_only else seq.ntok, H), generator=g).to(cuda)
    wf, wft = kernels.gemm_h_weight(gate_w), kernels.gemm_h_weight(gate_w.t().contiguous())
    # the three-launch reference
    xc_ref = kernels.conv_silu_fwd(x, conv_w, conv_b, seq=seq)
    rg_ref = kernels.gemm_nt_h(xc_ref, wf, 2 * H)
    _, car = kernels.gate_scan_fwd(rg_ref, xc_ref, z, lam, h0, gate_b=gate_b, seq=seq)
    dxz_ref = torch.empty_like(xz)
    drg_ref, dxc_ref, dlam_ref, dgb_ref, dh0_ref = kernels.gate_scan_bwd(
        rg_ref, xc_ref, z, lam, car, dy, dxz_ref[:, H:], gate_b=gate_b, seq=seq,
        last_only=last_only)
    dxc_g = kernels.gemm_nt_h(drg_ref, wft, H)
    dw_ref, db_ref = kernels.conv_silu_bwd(x, conv_w, conv_b, dxc_ref, dxc_g, dxz_ref[:, :H],
                                           seq=seq)
    # fused
    y, tc, *_ = kernels.grl_fwd(xz, conv_w, conv_b, wf, gate_b, lam, h0, seq,
                                want_y=not last_only, tile_carries=True)
    assert tc.shape == (seq.G, seq.max_tiles, H)
    out = kernels.grl_bwd(xz, conv_w, conv_b, wf, wft, gate_b, lam, h0, seq, tc, dy,
                          last_only=last_only, want_rmax=True)
    dxz, drg, xc, r_drg, r_xc, dlam, dgb, dh0, dw, db = out
    torch.cuda.synchronize()
    assert torch.equal(xc, xc_ref)
    for name, a, b in (("dz", dxz[:, H:], dxz_ref[:, H:]), ("dx", dxz[:, :H], dxz_ref[:, :H]),
                       ("drg", drg, drg_ref), ("dlam", dlam, dlam_ref),
                       ("dgate_b", dgb, dgb_ref), ("dh0", dh0, dh0_ref),
                       ("dconv_w", dw.reshape(-1), dw_ref.reshape(-1)), ("dconv_b", db, db_ref)):
        assert _rel(a, b) < 1e-5, (name, _rel(a, b))

    def gmax(t):
        m = torch.nn.functional.pad(t.abs().amax(1), (0, (-t.shape[0]) % 32)).view(-1, 32)
        return m.amax(1)

    assert torch.equal(r_xc, gmax(xc_ref))
    assert torch.equal(r_drg, gmax(drg))
    # deterministic
    out2 = kernels.grl_bwd(xz, conv_w, conv_b, wf, wft, gate_b, lam, h0, seq, tc, dy,
                           last_only=last_only, want_rmax=True)
    for a, b in zip(out, out2):
        assert torch.equal(a, b)


@pytest.mark.parametrize("packed_len", ["ragged", "fixed"])
def test_model_with_fused_forward_equals_three_launch(cuda, monkeypatch, packed_len):
    """RecBLR.calculate_loss + backward at d = 128 (H = 256): the fused
    forward and backward (default), the fused forward with the three-launch
    backward (RECBLR_FUSED_GRL_BWD=0) and RECBLR_FUSED_GRL=0 give the same
    loss and gradients within fp32 re-association, and the fused kernels
    ran."""
    from datamining_recblr_amd import kernels, recurrence
    from datamining_recblr_amd.distributed import synthetic_interaction
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset

    cfg = dict(hidden_size=128, loss_type="CE", num_layers=2, dropout_prob=0.0, expand=2,
               d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
               MAX_ITEM_LIST_LENGTH=200)
    torch.manual_seed(2020)
    model = RecBLR(cfg, SyntheticDataset(3000)).to(cuda).eval()
    inter = synthetic_interaction(256, 200, 3000, cuda, seed=9, fixed_len=packed_len == "fixed")
    calls = []
    orig = kernels.grl_fwd

    def counted(*a, **kw):
        calls.append(1)
        return orig(*a, **kw)

    monkeypatch.setattr(kernels, "grl_fwd", counted)
    bwd = []
    orig_b = kernels.grl_bwd
    monkeypatch.setattr(kernels, "grl_bwd", lambda *a, **k: bwd.append(1) or orig_b(*a, **k))
    res = {}
    for fused, fused_bwd in ((True, True), (True, False), (False, False)):
        monkeypatch.setattr(recurrence, "_FUSED", fused)
        monkeypatch.setattr(recurrence, "_FUSED_BWD", fused_bwd)
        calls.clear()
        bwd.clear()
        model.zero_grad(set_to_none=True)
        loss = model.calculate_loss(inter)
        loss.backward()
        res[fused, fused_bwd] = (loss.item(), {n: p.grad.clone() for n, p in model.named_parameters()
                                               if p.grad is not None})
        assert len(calls) == (2 if fused else 0), calls   # both layers
        assert len(bwd) == (2 if fused_bwd else 0), bwd
    ref = res[False, False]
    for key in ((True, True), (True, False)):
        assert abs(res[key][0] - ref[0]) < 1e-6 * max(1.0, abs(ref[0]))
        for n, gr in ref[1].items():
            err = (res[key][1][n] - gr).abs().max().item()
            assert err <= 1e-6 + 1e-5 * gr.abs().max().item(), (key, n, err)
