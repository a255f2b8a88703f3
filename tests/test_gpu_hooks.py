"""Module hooks on the HIP path (boundary fidelity): RecBole's
FLOP counter (get_flops, run.py:76-77) and profilers observe the model through
forward hooks on its nn.Linear / nn.Conv1d modules.  The in/out projections run
through their own nn.Linear __call__; the Linears and the conv fused into the
HIP kernels (gates, FeedForward w_1 / w_2, conv1d) fire their hooks with the
actual tensors.  Hooks only observe: the loss and every gradient are
bit-identical with and without them."""
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu


def _model_and_batch(cuda):
    from datamining_recblr_amd.distributed import synthetic_interaction
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset

    cfg = dict(hidden_size=64, loss_type="CE", num_layers=2, dropout_prob=0.0, expand=2,
               d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
               MAX_ITEM_LIST_LENGTH=50)
    torch.manual_seed(0)
    model = RecBLR(cfg, SyntheticDataset(300)).to(cuda)
    return model, synthetic_interaction(256, 50, 300, cuda, seed=1)


def _step(model, batch):
    model.zero_grad(set_to_none=True)
    loss = model.calculate_loss(batch)
    loss.backward()
    return loss.detach().clone(), {n: p.grad.clone() for n, p in model.named_parameters()
                                   if p.grad is not None}


def test_every_projection_and_conv_fires_its_hooks(cuda):
    model, batch = _model_and_batch(cuda)
    ref = _step(model, batch)
    seen = {}

    def hook(mod, args, out):
        seen.setdefault(mod, []).append((tuple(args[0].shape), tuple(out.shape)))
        if isinstance(mod, nn.Linear):
            x = args[0].reshape(-1, mod.in_features).double()
            want = x @ mod.weight.double().t()
            if mod.bias is not None:
                want = want + mod.bias.double()
            got = out.reshape(-1, mod.out_features).double()
            assert (got - want).abs().max().item() <= 1e-5 * (1 + want.abs().max().item())

    handles = [m.register_forward_hook(hook) for m in model.modules()
               if isinstance(m, (nn.Linear, nn.Conv1d))]
    try:
        got = _step(model, batch)
    finally:
        for h in handles:
            h.remove()
    mods = [m for m in model.modules() if isinstance(m, (nn.Linear, nn.Conv1d))]
    assert mods and all(m in seen for m in mods), [type(m).__name__ for m in mods if m not in seen]
    for m, calls in seen.items():
        for shp_in, shp_out in calls:
            if isinstance(m, nn.Linear):
                assert shp_in[-1] == m.in_features and shp_out[-1] == m.out_features
            else:
                assert shp_in[-2] == m.in_channels and shp_out[-2] == m.out_channels
    # observers only: bit-identical training step
    assert torch.equal(got[0], ref[0])
    for n, g in ref[1].items():
        assert torch.equal(got[1][n], g), n
    # a thop-style count over the Linears (RecBole's get_flops hook kind)
    flops = sum(shp_out_numel * m.in_features
                for m, calls in seen.items() if isinstance(m, nn.Linear)
                for shp_out_numel in [torch.Size(c[1]).numel() for c in calls])
    assert flops > 0
    assert type(model.recurrent_layers[0].behavior_modeling.input) is nn.Linear


def _hooked_layer_grads(cuda, defer, monkeypatch):
    """Tensor hooks on every RecurrentLayer output (dense batch, so each is
    [B, L, d] like the oracle's) and the oracle's gradients of the same
    tensors; with or without residual-gradient deferral."""
    from datamining_recblr_amd import blocks
    from datamining_recblr_amd.distributed import synthetic_interaction
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset
    from oracle import recblr_oracle as orc

    cfg = dict(hidden_size=64, loss_type="CE", num_layers=3, dropout_prob=0.0, expand=2,
               d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
               MAX_ITEM_LIST_LENGTH=50)
    monkeypatch.setattr(blocks, "_defer_residual", [defer])
    torch.manual_seed(0)
    model = RecBLR(cfg, SyntheticDataset(300)).to(cuda).eval()
    model.pack_sequences = False
    model.gather_last_layer = False
    batch = synthetic_interaction(16, 50, 300, cuda, seed=3)
    got = {}

    def fwd_hook(i):
        def hook(mod, args, out):
            out.register_hook(lambda g: got.__setitem__(i, g.detach().cpu().clone()))
        return hook

    hs = [layer.register_forward_hook(fwd_hook(i))
          for i, layer in enumerate(model.recurrent_layers)]
    try:
        model.calculate_loss(batch).backward()
    finally:
        for h in hs:
            h.remove()
    params = {k: v.detach().cpu().clone().requires_grad_(v.dtype.is_floating_point)
              for k, v in model.state_dict().items()}
    outs = []
    orig = orc.recurrent_layer_forward

    def rec(*a, **kw):
        h = orig(*a, **kw)
        h.retain_grad()
        outs.append(h)
        return h

    monkeypatch.setattr(orc, "recurrent_layer_forward", rec)
    cpu = {k: v.cpu() for k, v in batch.items()}
    orc.calculate_loss(params, cfg, cpu["item_id_list"], cpu["item_length"],
                       cpu["item_id"]).backward()
    want = {i: h.grad for i, h in enumerate(outs)}
    grads_ok = all(
        (p.grad.cpu() - params[n].grad).abs().max().item()
        <= 1e-4 + 1e-4 * params[n].grad.abs().max().item()
        for n, p in model.named_parameters() if params[n].grad is not None)
    return got, want, grads_ok


def test_tensor_hooks_see_full_gradient_without_deferral(cuda, monkeypatch):
    """RECBLR_DEFER_RESIDUAL=0 (blocks.set_defer_residual(False)): a tensor
    hook on a RecurrentLayer output (RecBLR.py:140-145) receives dL/dh of the
    reference, residual branch included, at 1e-4."""
    got, want, grads_ok = _hooked_layer_grads(cuda, False, monkeypatch)
    assert grads_ok
    assert sorted(got) == sorted(want) == [0, 1, 2]
    for i in want:
        err = (got[i] - want[i]).abs().max().item()
        assert err <= 1e-4 + 1e-4 * want[i].abs().max().item(), (i, err)


def test_deferred_residual_contract(cuda, monkeypatch):
    """Default (deferral on): parameter gradients are the reference's, the
    last layer's output gradient too (nothing downstream defers into it);
    an earlier layer's output hook sees the gradient WITHOUT the next
    layer's residual term — the documented contract."""
    got, want, grads_ok = _hooked_layer_grads(cuda, True, monkeypatch)
    assert grads_ok
    last = max(want)
    err = (got[last] - want[last]).abs().max().item()
    assert err <= 1e-4 + 1e-4 * want[last].abs().max().item()
    assert (got[0] - want[0]).abs().max().item() > 1e-3 * want[0].abs().max().item()


def test_modifying_hook_on_a_fused_linear_is_rejected(cuda):
    model, batch = _model_and_batch(cuda)
    h = model.recurrent_layers[0].ffn.w_1.register_forward_hook(lambda m, a, o: o * 2)
    try:
        with pytest.raises(NotImplementedError):
            model.calculate_loss(batch)
    finally:
        h.remove()


def test_parallel_scan_is_a_traceable_custom_op(cuda):
    """parallel_scan (the reference's kernel API) is the registered operator
    recblr::scan_fwd: torch.compile(fullgraph=True) traces forward and
    backward with no graph break, bit-identical to eager."""
    from datamining_recblr_amd.scan import parallel_scan

    g = torch.Generator().manual_seed(0)
    gates = (torch.rand(4, 32, 100, generator=g) * 0.1 + 0.9).to(cuda).requires_grad_(True)
    tokens = torch.randn(4, 32, 100, generator=g).to(cuda).requires_grad_(True)
    w = torch.randn(4, 32, 100, generator=g).to(cuda)

    def f(a, b):
        return (parallel_scan(a, b) * w).sum()

    ref = f(gates, tokens)
    ga, gb = torch.autograd.grad(ref, (gates, tokens))
    cf = torch.compile(f, fullgraph=True, backend="aot_eager")
    out = cf(gates, tokens)
    ca, cb = torch.autograd.grad(out, (gates, tokens))
    assert torch.equal(out, ref) and torch.equal(ca, ga) and torch.equal(cb, gb)


def test_linear_custom_op_transposed_input_compiles(cuda):
    """A non-contiguous (transposed) x through recblr::linear under
    torch.compile(fullgraph=True): the fake outputs' strides equal the real
    ones (contiguous), values and gradients equal eager's and fp64's."""
    from datamining_recblr_amd import ops

    g = torch.Generator().manual_seed(2)
    xt = torch.randn(128, 4500, generator=g).to(cuda)
    x = xt.t().requires_grad_(True)             # [4500, 128], strides (1, 4500)
    w = (torch.randn(256, 128, generator=g) * 0.05).to(cuda).requires_grad_(True)

    def f(x_, w_):
        return ops.linear(x_, w_, None).square().sum()

    eager = f(x, w)
    edx, edw = torch.autograd.grad(eager, (x, w))
    cf = torch.compile(f, fullgraph=True, backend="aot_eager")
    out = cf(x, w)
    dx, dw = torch.autograd.grad(out, (x, w))
    assert torch.equal(out, eager) and torch.equal(dx, edx) and torch.equal(dw, edw)
    xd, wd = x.detach().double(), w.detach().double()
    y = xd @ wd.t()
    for got, want in ((dx, 2 * y @ wd), (dw, 2 * y.t() @ xd)):
        assert ((got.double() - want).abs().max() / want.abs().max()).item() < 1e-5


def test_linear_custom_op_traces_and_matches(cuda):
    """recblr::linear (F.linear on the split-operand GEMMs) traces with
    torch.compile(fullgraph=True); value and dW against fp64."""
    from datamining_recblr_amd import ops

    g = torch.Generator().manual_seed(1)
    x = torch.randn(5000, 128, generator=g).to(cuda).requires_grad_(True)
    w = (torch.randn(512, 128, generator=g) * 0.05).to(cuda).requires_grad_(True)
    b = torch.randn(512, generator=g).to(cuda).requires_grad_(True)

    def f(x_, w_, b_):
        return ops.linear(x_, w_, b_).square().sum()

    cf = torch.compile(f, fullgraph=True, backend="aot_eager")
    out = cf(x, w, b)
    dx, dw, db = torch.autograd.grad(out, (x, w, b))
    xd, wd, bd = x.detach().double(), w.detach().double(), b.detach().double()
    y = xd @ wd.t() + bd
    assert abs(out.item() - y.square().sum().item()) <= 1e-5 * y.square().sum().item()
    for got, want in ((dx, 2 * y @ wd), (dw, 2 * y.t() @ xd), (db, 2 * y.sum(0))):
        assert ((got.double() - want).abs().max() / want.abs().max()).item() < 1e-5
