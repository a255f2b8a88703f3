"""Host-side logic that needs no GPU: padding arithmetic, the pad-prefix
closed form, module/parameter layout and init parity with the reference,
error behaviour."""
import pytest
import torch
import torch.nn.functional as F

from conftest import load_golden
from datamining_recblr_amd import RecBLRNativeError, kernels
from datamining_recblr_amd.distributed import shard_range, synthetic_interaction
from datamining_recblr_amd.model import GatedRecurrentLayer, RecBLR, lambda_init_range
from datamining_recblr_amd.recbole_compat import SyntheticDataset
from datamining_recblr_amd.recurrence import pad_prefix_state, pow2_pad_len
from oracle import recblr_oracle as orc


def test_pow2_pad_len_matches_reference_formula():
    for L in range(1, 5000):
        ref = 2 ** ((L - 1).bit_length()) - L      # RecBLR.py:177
        assert pow2_pad_len(L) == ref
        T = L + ref
        assert T & (T - 1) == 0 and T >= L


@pytest.mark.parametrize("P", [1, 14, 56, 1000])
def test_pad_prefix_closed_form_matches_serial_pad_steps(P):
    """h after P pad steps == running the reference's padded recurrence on the
    constant pad inputs (value and parameter gradients)."""
    torch.manual_seed(P)
    H = 32
    conv_b = (torch.randn(H) * 2).requires_grad_()
    gw = (torch.randn(2 * H, H) * 0.2).requires_grad_()
    gb = torch.randn(2 * H).requires_grad_()
    lo, hi = lambda_init_range()
    lam = torch.linspace(lo, hi, H).requires_grad_()
    h0 = pad_prefix_state(conv_b, gw, gb, lam, P)
    (h0 * torch.arange(H)).sum().backward()
    g1 = [t.grad.clone() for t in (conv_b, gw, gb, lam)]
    for t in (conv_b, gw, gb, lam):
        t.grad = None
    # pad-step constants in fp32 exactly as the reference computes them
    # (RecBLR.py:185,196-199 on an all-zero padded input), then the P serial
    # recurrence steps in fp64 so only the closed form itself is under test
    xc = F.silu(conv_b)
    r, i = (xc @ gw.t() + gb).chunk(2)
    a = torch.exp(-F.softplus(lam) * torch.sigmoid(r))
    bp = torch.sqrt(1 - a.pow(2) + 1e-8) * torch.sigmoid(i) * xc
    a, bp = a.double(), bp.double()
    h = torch.zeros(H, dtype=torch.float64)
    for _ in range(P):
        h = a * h + bp
    (h * torch.arange(H)).sum().backward()
    # fp32 rounding of alpha compounds over P steps: ~P * 6e-8 relative
    torch.testing.assert_close(h0.detach().double(), h.detach(), atol=1e-5, rtol=5e-5)
    for ga, t in zip(g1, (conv_b, gw, gb, lam)):
        torch.testing.assert_close(ga, t.grad, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("idx", range(6))
def test_init_and_state_dict_parity_with_reference(idx):
    """Same seed -> bit-identical initial weights and identical state_dict keys."""
    case = load_golden("model_golden.pt")[idx]
    torch.manual_seed(2020)
    model = RecBLR(case["cfg"], SyntheticDataset(case["n_items"]))
    sd = model.state_dict()
    assert list(sd.keys()) == list(case["init_state"].keys())
    for k, v in case["init_state"].items():
        assert torch.equal(sd[k], v), k


def test_lambda_init_range():
    lo, hi = lambda_init_range()
    sp = F.softplus(torch.tensor([lo, hi]))
    torch.testing.assert_close(torch.exp(-sp), torch.tensor([0.9, 0.999]))


def test_cpu_forward_fails_loudly():
    layer = GatedRecurrentLayer(d_model=16)
    with pytest.raises(RecBLRNativeError):
        layer(torch.randn(2, 5, 16))
    with pytest.raises(RecBLRNativeError):
        kernels.scan_fwd(torch.rand(1, 2, 3), torch.rand(1, 2, 3))
    with pytest.raises(RecBLRNativeError):
        kernels.gate_scan_fwd(torch.rand(1, 2, 8), torch.rand(1, 2, 4), torch.rand(1, 2, 4),
                              torch.rand(4))


def test_bad_loss_type():
    cfg = dict(hidden_size=16, loss_type="XX", num_layers=1, dropout_prob=0.1, expand=2, d_conv=4,
               bd_lru_only=False, disable_conv1d=False, disable_ffn=False, MAX_ITEM_LIST_LENGTH=10)
    with pytest.raises(NotImplementedError):
        RecBLR(cfg, SyntheticDataset(10))


def test_bd_lru_only_implies_flags():
    cfg = dict(hidden_size=16, loss_type="CE", num_layers=2, dropout_prob=0.1, expand=2, d_conv=4,
               bd_lru_only=True, disable_conv1d=False, disable_ffn=False, MAX_ITEM_LIST_LENGTH=10)
    m = RecBLR(cfg, SyntheticDataset(10))
    assert m.disable_conv1d and m.disable_ffn
    assert all(layer.disable_ffn for layer in m.recurrent_layers)
    assert all(layer.behavior_modeling.disable_conv1d for layer in m.recurrent_layers)


def test_recbole_field_names():
    cfg = dict(hidden_size=16, loss_type="CE", num_layers=1, dropout_prob=0.1, expand=2, d_conv=4,
               bd_lru_only=False, disable_conv1d=False, disable_ffn=False, MAX_ITEM_LIST_LENGTH=10)
    m = RecBLR(cfg, SyntheticDataset(10))
    assert (m.ITEM_SEQ, m.ITEM_SEQ_LEN, m.POS_ITEM_ID, m.NEG_ITEM_ID, m.ITEM_ID) == \
        ("item_id_list", "item_length", "item_id", "neg_item_id", "item_id")
    out = torch.arange(2 * 5 * 3, dtype=torch.float32).view(2, 5, 3)
    assert torch.equal(m.gather_indexes(out, torch.tensor([0, 4])), out[[0, 1], [0, 4]])


def test_shard_range_and_synthetic_batch():
    for n in (1, 7, 2048, 16384):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    inter = synthetic_interaction(16, 20, 50, "cpu", seed=0, with_neg=True)
    seq, lens = inter["item_id_list"], inter["item_length"]
    assert seq.shape == (16, 20) and lens.min() >= 1 and lens.max() <= 20
    for b in range(16):
        assert (seq[b, :lens[b]] > 0).all() and (seq[b, lens[b]:] == 0).all()


def test_oracle_scan_reverse_matches_autograd_of_loop():
    """SerialScan.backward (the reference's glue, parallel_scan.py:106-113) ==
    autograd through the plain serial loop."""
    torch.manual_seed(0)
    g = torch.rand(2, 3, 17).requires_grad_()
    x = torch.randn(2, 3, 17).requires_grad_()
    gy = torch.randn(2, 3, 17)
    orc.oracle_parallel_scan(g, x).backward(gy)
    g2 = g.detach().clone().requires_grad_()
    x2 = x.detach().clone().requires_grad_()
    h = torch.zeros(2, 3)
    outs = []
    for t in range(17):
        h = h * g2[..., t] + x2[..., t]
        outs.append(h)
    torch.stack(outs, -1).backward(gy)
    torch.testing.assert_close(g.grad, g2.grad)
    torch.testing.assert_close(x.grad, x2.grad)


def test_tuned_gemm_table_covers_bench_shapes():
    """The shipped TunableOp table is well-formed and lists the C2 projection
    GEMMs (B*L = 409,600 rows; K, N in {128, 256, 512})."""
    import csv

    from datamining_recblr_amd import gemm_tuning

    rows = list(csv.reader(open(gemm_tuning.TABLE_PATH)))
    validators = {r[1]: r[2] for r in rows if r[0] == "Validator"}
    assert validators["GCN_ARCH_NAME"].startswith("gfx950")
    assert "PT_VERSION" in validators and "HIPBLASLT_VERSION" in validators
    entries = [r for r in rows if r[0] != "Validator"]
    assert entries and all(len(r) == 4 and float(r[3]) > 0 for r in entries)
    keys = " ".join(r[1] for r in entries)
    for shape in ("512_409600_128", "512_409600_256", "128_409600_256", "128_409600_512"):
        assert shape in keys
    assert gemm_tuning.use_tuned_gemms() is False or torch.cuda.is_available()


def test_tuned_gemm_table_lists_the_configs4_library_shapes():
    """The table also carries the configs[4] GEMMs the per-shape bf16 mode
    leaves on the library (round 5's TunableOp search): the K = 1,024 input
    gradients and the three weight gradients' batched products, bf16."""
    import csv

    from datamining_recblr_amd import gemm_tuning

    rows = [r for r in csv.reader(open(gemm_tuning.TABLE_PATH)) if r[0] != "Validator"]
    bf16 = {r[1] for r in rows if "BFloat16" in r[0]}
    for key in ("nn_512_2097152_1024", "nn_256_2097152_1024", "nt_512_256_32768_B_64",
                "nt_512_1024_32768_B_64", "nt_256_1024_32768_B_64"):
        assert any(k.startswith(key) for k in bf16), key
    assert len({(r[0], r[1]) for r in rows}) == len(rows)   # no duplicate keys


def test_bf16_gemm_modes_and_shape_rule(monkeypatch):
    """RECBLR_BF16_GEMM: set_bf16_gemm takes "auto" / "1" / "0" or a bool and
    returns the previous mode; anything else is rejected.  In "auto" only the
    NT GEMMs with R <= 512 inputs run on our kernels, no weight gradient."""
    from datamining_recblr_amd import linear

    prev = linear.set_bf16_gemm("auto")
    try:
        assert linear.set_bf16_gemm(True) == "auto"
        assert linear.set_bf16_gemm(False) == "1"
        assert linear.set_bf16_gemm("auto") == "0"
        with pytest.raises(ValueError):
            linear.set_bf16_gemm("yes")
        assert linear._bf16_gemm == "auto"
        assert linear.BF16_NT_MAX_R == 512
        assert linear.BF16_NT_MIN_ROWS == 65536
    finally:
        linear.set_bf16_gemm(prev)


def test_rank_metrics_match_sklearn_and_recbole():
    """rank_metrics from (n_greater, n_equal) equals sklearn's tie-averaged
    ndcg_score (run_with_unseen.py:247) and RecBole-style top-k metrics on an
    explicit score matrix with ties."""
    from sklearn.metrics import ndcg_score

    from datamining_recblr_amd.scoring import rank_metrics

    g = torch.Generator().manual_seed(0)
    B, V = 64, 40
    scores = torch.randint(0, 12, (B, V), generator=g).double()  # many ties
    tgt = torch.randint(0, V, (B,), generator=g)
    ts = scores[torch.arange(B), tgt]
    others = torch.ones(B, V, dtype=torch.bool)
    others[torch.arange(B), tgt] = False
    gt = ((scores > ts[:, None]) & others).sum(1)
    eq = ((scores == ts[:, None]) & others).sum(1)
    y = torch.zeros(B, V)
    y[torch.arange(B), tgt] = 1
    for k in (5, 10):
        ref = ndcg_score(y.numpy(), scores.numpy(), k=k)
        m = rank_metrics(gt, eq, topk=(k,), ties="average")
        assert abs(m[f"ndcg@{k}"] - ref) < 1e-12
    # optimistic ranks: exact RecBole metrics when the target wins its ties
    order = torch.argsort(-(scores + 1e-6 * (~others).double()), dim=1, stable=True)
    pos = (order == tgt[:, None]).double().argmax(1).double()
    m = rank_metrics(gt, eq, topk=(10,))
    assert abs(m["hit@10"] - (pos < 10).double().mean().item()) < 1e-12
    assert abs(m["mrr@10"] - torch.where(pos < 10, 1 / (pos + 1.0), 0.0).mean().item()) < 1e-12
    ndcg = torch.where(pos < 10, 1 / torch.log2(pos + 2.0), 0.0).mean().item()
    assert abs(m["ndcg@10"] - ndcg) < 1e-12
    # invalid rows (-1) are dropped
    m2 = rank_metrics(torch.cat([gt, torch.tensor([-1])]), None, topk=(10,))
    assert abs(m2["hit@10"] - m["hit@10"]) < 1e-12


def test_split_cache_counts_optimizer_steps():
    """The split-weight cache (linear._weight_split) is invalidated by every
    torch.optim step through the global step hook, whatever the optimizer
    does to the version counters."""
    import torch

    from datamining_recblr_amd import linear

    w = torch.nn.Parameter(torch.randn(4, 4))
    opt = torch.optim.SGD([w], lr=0.1)
    n0 = linear._opt_steps[0]
    w.grad = torch.ones(4, 4)
    opt.step()
    assert linear._opt_steps[0] == n0 + 1


def test_custom_op_fakes_are_contiguous_like_the_real_outputs():
    """torch.compile / export trace the ops through their fake impls: the
    fakes must give the real outputs' strides (contiguous) even for a
    transposed input, or a compiled graph would assume a wrong layout."""
    from torch._subclasses.fake_tensor import FakeTensorMode

    from datamining_recblr_amd import ops

    with FakeTensorMode():
        x = torch.empty(128, 300).t()          # [300, 128], strides (1, 300)
        w = torch.empty(64, 128)
        dy = torch.empty(300, 64)
        dx, dw, db = ops.linear_bwd(dy, x, w, True)
        y = ops.linear(x, w, None)
        g = torch.empty(2, 4, 9)
        s = ops.scan_fwd(g, g)
        dg, dt = ops.scan_bwd(g, s, g)
    assert dx.shape == x.shape and dx.is_contiguous() and not x.is_contiguous()
    assert dw.shape == w.shape and dw.is_contiguous() and db.shape == (64,)
    assert y.shape == (300, 64) and y.is_contiguous()
    assert s.is_contiguous() and dg.is_contiguous() and dt.is_contiguous()


def test_interaction_to_keeps_host_lengths():
    """run.py's Trainer moves each CPU batch with Interaction.to(device)
    (RecBole); the stand-in (and the hook installed on RecBole's class) keeps
    the host copy of item_length on the moved tensor, so the packed forward
    needs no device sync for the token count."""
    from datamining_recblr_amd.model import HOST_LENGTHS
    from datamining_recblr_amd.recbole_compat import Interaction

    lengths = torch.tensor([3, 1, 7])
    inter = Interaction({"item_id_list": torch.zeros(3, 7, dtype=torch.int64),
                         "item_length": lengths, "item_id": torch.ones(3, dtype=torch.int64)})
    moved = inter.to("meta")
    assert moved["item_length"].device.type == "meta"
    assert torch.equal(getattr(moved["item_length"], HOST_LENGTHS), lengths)
    assert not hasattr(moved["item_id"], HOST_LENGTHS)
    # a CPU -> CPU move attaches nothing (the tensor is already on the host)
    assert not hasattr(inter.to("cpu")["item_length"], HOST_LENGTHS)


@pytest.mark.parametrize("cus", [80, 104, 228, 256, 304])
def test_ce_weight_gradient_splits_are_multiples_of_8(monkeypatch, cus):
    """The CE backward's row splits for rb_gemm_tn_h (multiples of 8, >= 8)
    on any CU count and batch: B = 768 / 1792 on 256 CUs and B = 2048 on a
    304-CU part gave 84 / 36 / 36 before the rounding."""
    from datamining_recblr_amd import linear, scoring

    monkeypatch.setitem(linear._ncus, "fake", cus)
    for B in (256, 512, 768, 1792, 2048, 4096):
        for V in (500, 10544, 65536):
            nt1 = ((V + 255) // 256) * 1
            s1 = max(8, min(scoring._tn_splits8("fake", nt1), B // 256 // 8 * 8))
            s2 = scoring._tn_splits8("fake", (B // 256) * 1, div=2)
            assert s1 % 8 == 0 and s1 >= 8, (B, V, s1)
            assert s2 % 8 == 0 and s2 >= 8, (B, V, s2)


def test_ce_f16_grads_fall_back_past_the_weight_gradient_width(monkeypatch):
    """The f16 CE backward (RECBLR_CE_GRADS=f16) runs the item gradient as
    rb_gemm_tn_h with N = V rounded up to 256 <= 65536; larger vocabularies
    take the sliced path instead of failing in the kernel."""
    from datamining_recblr_amd import linear, scoring

    if linear.gemm_format() != "f16x3":
        pytest.skip("f16x3 GEMMs not selected in this environment")
    monkeypatch.setattr(scoring, "CE_GRADS", "f16")
    seq = torch.empty(256, 128)
    assert scoring._f16_grads_ok(seq, torch.empty(65536, 128))
    assert not scoring._f16_grads_ok(seq, torch.empty(65537, 128))
    assert not scoring._f16_grads_ok(torch.empty(300, 128), torch.empty(1000, 128))


def test_bit31_placement_keeps_the_whole_run_in_an_upper_half():
    """tests/placement.bit31_offset (the GPU tests' operands above bit 31):
    every byte of the run has bit 31 set and stays inside the allocation,
    for allocation bases anywhere in a 4 GiB block, including bases whose
    upper half is too short for the run."""
    import random

    from tests.placement import bit31_alloc_bytes, bit31_offset

    rng = random.Random(31)
    need = 4 * 204632 * (512 + 256) + 512
    bases = [k * 256 for k in (0, 1)] + [(1 << 31) - 256, 1 << 31, (1 << 32) - 256,
                                         (1 << 32) - need // 2 // 256 * 256]
    bases += [rng.randrange(0, 1 << 47) // 256 * 256 for _ in range(2000)]
    for base in bases:
        off = bit31_offset(base, need)
        a, end = base + off, base + off + need - 1
        assert a % 256 == 0
        assert (a >> 31) & 1 and (end >> 31) & 1 and (a >> 32) == (end >> 32), hex(base)
        assert off + need <= bit31_alloc_bytes(need)


def test_ce_env_switches_are_checked(monkeypatch):
    """RECBLR_CE_* switches are validated at import: an unknown value (e.g. the
    removed CE_GRADS=fused) raises instead of silently choosing a slower
    path, as RECBLR_GEMM / RECBLR_BF16_GEMM do."""
    from datamining_recblr_amd import scoring

    monkeypatch.setenv("RECBLR_CE_GRADS", "fused")
    with pytest.raises(ValueError, match="RECBLR_CE_GRADS"):
        scoring._env_choice("RECBLR_CE_GRADS", "f16", ("f16", "torch"))
    monkeypatch.setenv("RECBLR_CE_GRADS", "torch")
    assert scoring._env_choice("RECBLR_CE_GRADS", "f16", ("f16", "torch")) == "torch"
    monkeypatch.delenv("RECBLR_CE_GRADS")
    assert scoring._env_choice("RECBLR_CE_GRADS", "f16", ("f16", "torch")) == "f16"
