"""End-to-end parity of the configurations the benchmark times, with the
f16x3 projection GEMMs (csrc/gemm_half.hip: rb_gemm_nt_h forward / input
gradients, rb_gemm_tn_h weight gradients) asserted engaged.

RecBLR.calculate_loss + backward (RecBLR.py:86-103, 210-227 and the encoder
:75-84, :140-207) on the GPU against the CPU oracle (oracle/recblr_oracle.py,
pinned to the reference's own outputs by tests/test_oracle_golden.py): the
loss and every parameter gradient at 1e-4 (abs + rel, plus 2e-6 of the
tensor's max for fp32 re-association over long reductions).

Shapes:
* C2 (BASELINE configs[1]/[3] per GPU): d = 128, L = 200, n_items = 10,544 —
  B = 64 (ntok ~ 6.5k packed, 12.8k dense: above the split kernel's row
  threshold, so the bench's own routing is exercised);
* C3 (configs[2], amazon-beauty shape; the dataset is absent, synthetic
  stand-in): d = 128, L = 50, B = 2048 (train_batch_size), n_items = 10,544.
Each runs packed (the benchmark's default) and dense; every projection, the
gathered last-layer tail included, runs on the split kernels.  Eval mode: dropout streams differ
between implementations.
"""
import pytest
import torch

from oracle import recblr_oracle as orc

pytestmark = pytest.mark.gpu

N_ITEMS = 10544


def close(a, b, atol=1e-4, rtol=1e-4, what=""):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    err = (a - b).abs()
    bad = err > atol + rtol * b.abs() + 2e-6 * b.abs().max()
    assert not bad.any(), f"{what}: max err {err.max().item():.3e} (max |ref| {b.abs().max():.3e})"


def _cfg(L, loss_type="CE", d=128):
    return dict(hidden_size=d, loss_type=loss_type, num_layers=2, dropout_prob=0.2, expand=2,
                d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
                MAX_ITEM_LIST_LENGTH=L)


def _run(cuda, B, L, packed, gather, seed, loss_type="CE", fixed_len=False):
    from datamining_recblr_amd.distributed import synthetic_interaction
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset

    cfg = _cfg(L, loss_type)
    torch.manual_seed(2020)
    model = RecBLR(cfg, SyntheticDataset(N_ITEMS)).to(cuda).eval()
    model.pack_sequences, model.gather_last_layer = packed, gather
    inter = synthetic_interaction(B, L, N_ITEMS, cuda, seed=seed, with_neg=loss_type == "BPR",
                                  fixed_len=fixed_len)
    loss = model.calculate_loss(inter)
    loss.backward()
    torch.cuda.synchronize()
    params = {k: v.detach().cpu().clone().requires_grad_(v.dtype.is_floating_point)
              for k, v in model.state_dict().items()}
    cpu = {k: v.cpu() for k, v in inter.items()}
    ref = orc.calculate_loss(params, cfg, cpu["item_id_list"], cpu["item_length"],
                             cpu["item_id"], cpu.get("neg_item_id"))
    ref.backward()
    close(loss, ref, what="loss")
    for n, p in model.named_parameters():
        close(p.grad, params[n].grad, what=f"d{n}")
    return int(cpu["item_length"].sum())


@pytest.mark.parametrize("packed", [True, False], ids=["packed", "dense"])
@pytest.mark.parametrize("B,L", [(64, 200), (2048, 50)], ids=["C2", "C3"])
def test_train_step_matches_oracle_with_split_gemm(cuda, split_gemm_calls, monkeypatch, B, L,
                                                   packed):
    from datamining_recblr_amd import kernels, recurrence

    fused, fused_b = [], []
    orig, orig_b = kernels.grl_fwd, kernels.grl_bwd
    monkeypatch.setattr(kernels, "grl_fwd", lambda *a, **k: fused.append(1) or orig(*a, **k))
    monkeypatch.setattr(kernels, "grl_bwd", lambda *a, **k: fused_b.append(1) or orig_b(*a, **k))
    ntok = _run(cuda, B, L, packed, True, seed=B + L)
    rows = ntok if packed else B * L
    big = [c for c in split_gemm_calls if c[0] == rows]
    # per layer and direction: in, gates, out (fwd) and their dX GEMMs; layer
    # 0's FFN (the last layer's tail runs on the B gathered rows).  Packed,
    # with RECBLR_FUSED_GRL=1 (opt-in, off by default) the gates forward GEMM
    # runs inside rb_grl_fwd, and with RECBLR_FUSED_GRL_BWD=1 the gates dX
    # GEMM inside rb_grl_bwd.
    on = packed and recurrence._FUSED
    on_b = on and recurrence._FUSED_BWD
    assert len(big) >= 12 - 2 * on - 2 * on_b, (rows, split_gemm_calls)
    shapes = {(c[1], c[2]) for c in big}
    for s in ((128, 512), (256, 128), (512, 128), (128, 256)):
        assert s in shapes, (s, shapes)
    assert len(fused) == 2 * on and len(fused_b) == 2 * on_b, (fused, fused_b)
    assert ((256, 512) in shapes) != on and ((512, 256) in shapes) != on_b, shapes
    assert any(c[0] == B for c in split_gemm_calls), "gathered tail not on the kernel"


@pytest.mark.parametrize("fixed_len", [False, True], ids=["ragged", "fixed_len"])
def test_timed_shape_weight_gradients_on_tn_kernel(cuda, split_gemm_calls, tn_gemm_calls,
                                                   fixed_len):
    """The bench's shape (d = 128, L = 200, n_items = 10,544, packed, gathered
    tail) at B = 192: ntok >= linear.MIN_ROWS_FOR_SPLIT, so every [ntok]-row
    weight gradient (RecBLR.py:162,165,167,213,214) runs on rb_gemm_tn_h with
    the rmax side outputs of the forward / input-gradient GEMMs — the
    configuration the benchmark times — and loss plus every gradient match
    the oracle at 1e-4.  fixed_len: every sequence of length 200 (the bench's
    fixed_length companion)."""
    from datamining_recblr_amd import linear

    B, L = 192, 200
    ntok = _run(cuda, B, L, packed=True, gather=True, seed=11, fixed_len=fixed_len)
    assert ntok >= linear.MIN_ROWS_FOR_SPLIT, ntok
    big = [c for c in tn_gemm_calls if c[0] == ntok]
    # layer 0: input, gates, output, w_1, w_2; layer 1: input, gates (its
    # output projection and FFN run on the B gathered rows)
    shapes = sorted((c[1], c[2]) for c in big)
    assert len(big) >= 7, tn_gemm_calls
    for s in ((512, 128), (512, 256), (128, 256), (512, 128), (128, 512)):
        assert s in shapes, (s, shapes)
    assert any(c[0] == ntok for c in split_gemm_calls)


def test_all_positions_tail_matches_oracle(cuda, split_gemm_calls):
    """C2 dense with the last layer's tail at every position (the reference's
    arithmetic, RECBLR_FULL_LAST_LAYER=1): both FFNs on B*L rows."""
    B, L = 64, 200
    _run(cuda, B, L, packed=False, gather=False, seed=7)
    assert sum(1 for c in split_gemm_calls if c == (B * L, 128, 512)) >= 6


def test_bpr_c3_matches_oracle(cuda, split_gemm_calls):
    """BPR loss (RecBLR.py:89-95) at the C3 shape, packed."""
    _run(cuda, 2048, 50, packed=True, gather=True, seed=5, loss_type="BPR")
    assert len(split_gemm_calls) >= 12


@pytest.mark.experimental
@pytest.mark.parametrize("bwd", [False, True], ids=["fused_fwd", "fused_fwd_bwd"])
@pytest.mark.parametrize("B,L", [(192, 200), (2048, 50)], ids=["C2", "C3"])
def test_fused_grl_kernels_match_oracle(cuda, monkeypatch, B, L, bwd):
    """The opt-in one-launch GatedRecurrentLayer kernels (rb_grl_fwd, and
    rb_grl_bwd with bwd; RECBLR_FUSED_GRL / RECBLR_FUSED_GRL_BWD) in the whole
    training step against the CPU oracle — loss and every parameter gradient
    at the suite's 1e-4 bar — with both kernels asserted engaged on both
    layers (tests/test_gpu_fused.py compares them with the three-launch path)."""
    from datamining_recblr_amd import kernels, recurrence

    monkeypatch.setattr(recurrence, "_FUSED", True)
    monkeypatch.setattr(recurrence, "_FUSED_BWD", bwd)
    fwd_calls, bwd_calls = [], []
    orig, orig_b = kernels.grl_fwd, kernels.grl_bwd
    monkeypatch.setattr(kernels, "grl_fwd", lambda *a, **k: fwd_calls.append(1) or orig(*a, **k))
    monkeypatch.setattr(kernels, "grl_bwd", lambda *a, **k: bwd_calls.append(1) or orig_b(*a, **k))
    _run(cuda, B, L, packed=True, gather=True, seed=B + 3 * L)
    assert len(fwd_calls) == 2 and len(bwd_calls) == 2 * bwd, (fwd_calls, bwd_calls)
