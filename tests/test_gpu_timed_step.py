"""The exact training step bench.py times, end to end against the oracle.

bench.py's headline (BASELINE.json metric): RecBLR
calculate_loss (CE over n_items = 10,544) + backward at B = 2048, L = 200,
d = 128, two layers, packed sequences, the last layer's position-wise tail on
the gathered rows — on bench.py's own synthetic batches
(`synthetic_interaction(2048, 200, 10544, seed=0)` is the first of its four
batches, `seed=50, fixed_len=True` the first of its `fixed_length` companion's).
At ntok ~ 204k packed rows every size-dependent piece runs at the size the
benchmark times: the persistent NT tiles plus the 256 x 64 tail phase of
rb_gemm_nt_h, the row-chunk scales and split count of rb_gemm_tn_h, the CE's
vocabulary splits and its two-layout gradient on the f16 pipe.  All asserted
engaged below.

The oracle (oracle/recblr_oracle.py, pinned to the reference's own outputs by
tests/test_oracle_golden.py; RecBLR.py:75-103, 140-227, parallel_scan.py:83-114)
runs on the device's copies of the same parameters and inputs in fp32 torch
ops (hipBLASLt GEMMs, serial scan): a CPU run of this size takes minutes.
MIOpen is switched off for it, so its depthwise conv is torch's own kernel.

Eval mode (dropout off): the dropout streams of the two implementations
cannot match mask for mask.  Bar: the suite's 1e-4 abs + 1e-4
rel, plus 2e-6 of the tensor's max for fp32 re-association over ~204k-row
reductions.
"""
import pytest
import torch

from oracle import recblr_oracle as orc

pytestmark = pytest.mark.gpu

B, L, D, N_ITEMS = 2048, 200, 128, 10544


def close(a, b, atol=1e-4, rtol=1e-4, what=""):
    a, b = a.detach().float(), b.detach().float()
    err = (a - b).abs()
    bad = err > atol + rtol * b.abs() + 2e-6 * b.abs().max()
    assert not bad.any(), (f"{what}: max err {err.max().item():.3e} "
                           f"(max |ref| {b.abs().max().item():.3e}, {int(bad.sum())} bad)")


def _cfg():
    return dict(hidden_size=D, loss_type="CE", num_layers=2, dropout_prob=0.2, expand=2,
                d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
                MAX_ITEM_LIST_LENGTH=L)


@pytest.mark.parametrize("seed,fixed_len", [(0, False), (50, True)], ids=["ragged", "fixed_len"])
def test_bench_step_matches_oracle(cuda, split_gemm_calls, tn_gemm_calls, seed, fixed_len):
    from datamining_recblr_amd import kernels
    from datamining_recblr_amd.distributed import synthetic_interaction
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset

    cfg = _cfg()
    torch.manual_seed(2020)   # bench.py's model seed
    model = RecBLR(cfg, SyntheticDataset(N_ITEMS)).to(cuda).eval()
    assert model.pack_sequences and model.gather_last_layer   # the bench's defaults
    inter = synthetic_interaction(B, L, N_ITEMS, cuda, seed=seed, fixed_len=fixed_len)
    ntok = int(inter["item_length"].sum())
    with kernels.kernel_timing() as t:
        loss = model.calculate_loss(inter)
        loss.backward()
    torch.cuda.synchronize()
    names = {r[0] for r in t.records}

    # --- the size-dependent kernels ran at the bench's row count ---
    assert ntok > (200_000 if not fixed_len else B * L - 1), ntok
    nt_big = [c for c in split_gemm_calls if c[0] == ntok]
    # layer 0: in, gates, out, w_1, w_2 forward + their dX (w_1's via the
    # fused activation epilogue); layer 1: in, gates forward + dX
    assert len(nt_big) >= 12, split_gemm_calls
    assert {(128, 512), (256, 512), (256, 128), (128, 256), (512, 128), (512, 256)} <= \
        {(c[1], c[2]) for c in nt_big}, nt_big
    tn_big = [c for c in tn_gemm_calls if c[0] == ntok]
    assert len(tn_big) >= 7, tn_gemm_calls
    assert any(c[0] == B for c in tn_gemm_calls), "CE gradient products not on rb_gemm_tn_h"
    assert {"rb_item_split_h", "rb_item_ce_fwd_h"} <= names, names
    assert names & {"rb_item_ce_probs_h", "rb_item_ce_probs_h_both"}, names
    assert {"rb_gate_scan_fwd", "rb_gate_scan_bwd", "rb_conv_silu_bwd"} <= names, names

    # --- the oracle on the same parameters and batch ---
    params = {k: v.detach().clone().requires_grad_(v.dtype.is_floating_point)
              for k, v in model.state_dict().items()}
    prev = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False
    try:
        ref = orc.calculate_loss(params, cfg, inter["item_id_list"], inter["item_length"],
                                 inter["item_id"])
        ref.backward()
    finally:
        torch.backends.cudnn.enabled = prev
    torch.cuda.synchronize()
    close(loss, ref, what="loss")
    for n, p in model.named_parameters():
        close(p.grad, params[n].grad, what=f"d{n}")
