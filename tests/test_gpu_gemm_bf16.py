"""bf16-operand projection GEMMs (csrc/gemm_bf16.hip: rb_gemm_nt_bf16,
rb_gemm_bf16_weight_image) — the configs[4] Linears (RecBLR.py:162,165,167
and their autograd) on bf16 activations; their weight gradients run on
hipBLASLt's split-K (round 5's rb_gemm_tn_bf16 was removed in round 6).

Reference: the same bf16 operands in fp64 on the host.  The NT output is one
rounding of an fp32 sum to bf16, so each element must sit within a bf16
half-ulp (2^-9 relative, tested at 2^-8) plus the fp32 accumulation bound
(K 2^-24 sum |a w|, tested at 1e-5 of that sum)."""
import pytest
import torch

from datamining_recblr_amd import kernels, linear
from tests.placement import bit31_alloc_bytes, bit31_offset

BF = torch.bfloat16
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    return torch.device("cuda:0")


def _nt_ref(a, wb, bias):
    ref = a.double().cpu() @ wb.double().cpu().t()
    mag = a.double().abs().cpu() @ wb.double().abs().cpu().t()
    if bias is not None:
        ref = ref + bias.double().cpu()
        mag = mag + bias.double().abs().cpu()
    return ref, mag


@pytest.mark.parametrize("M,R,C,with_bias", [
    (4096 + 37, 256, 1024, True),     # in-proj shape, partial last row tile
    (2048, 512, 1024, True),          # gates
    (1000, 512, 256, False),          # out-proj, fewer rows than one round
    (300, 64, 512, False),            # one k-step per tile (stores flushed per tile)
    (8 * 256 * 3 + 5, 1024, 512, False),   # dX shapes: K = 1024
])
def test_gemm_nt_bf16_vs_fp64(cuda, M, R, C, with_bias):
    g = torch.Generator(device=cuda).manual_seed(M + R + C)
    a = torch.randn(M, R, device=cuda, generator=g).to(BF)
    w = torch.randn(C, R, device=cuda, generator=g) * R ** -0.5
    bias = torch.randn(C, device=cuda, generator=g) if with_bias else None
    out = kernels.gemm_nt_bf16(a, kernels.bf16_weight_image(w), C, bias=bias)
    assert out.dtype == BF and out.shape == (M, C)
    ref, mag = _nt_ref(a, w.to(BF), bias)
    err = (out.double().cpu() - ref).abs()
    bound = 2.0 ** -8 * ref.abs() + 1e-5 * mag + 1e-30
    assert bool((err <= bound).all()), f"max excess {(err - bound).max().item():.3e}"


def test_gemm_nt_bf16_transposed_image(cuda):
    """The input-gradient form dX = dY W: Bm = W^T from the transposed image."""
    g = torch.Generator(device=cuda).manual_seed(3)
    M, N, K = 4096, 1024, 256            # dY [M, N], W [N, K] -> dX [M, K]
    dy = torch.randn(M, N, device=cuda, generator=g).to(BF)
    w = torch.randn(N, K, device=cuda, generator=g) * N ** -0.5
    out = kernels.gemm_nt_bf16(dy, kernels.bf16_weight_image(w, transpose=True), K)
    ref, mag = _nt_ref(dy, w.to(BF).t(), None)
    err = (out.double().cpu() - ref).abs()
    assert bool((err <= 2.0 ** -8 * ref.abs() + 1e-5 * mag).all())


def test_bf16_weight_image_layout(cuda):
    """Fragment (cb, kb), lane l: column 16 cb + l % 16, k 32 kb + 8 (l / 16) + j."""
    C, R = 64, 96
    w = torch.arange(C * R, device=cuda, dtype=torch.float32).view(C, R) / 64.0
    img = kernels.bf16_weight_image(w).view(C // 16, R // 32, 64, 8).cpu()
    wb = w.to(BF).cpu()
    for cb in range(C // 16):
        for kb in range(R // 32):
            for lane in (0, 5, 15, 16, 31, 47, 63):
                c, k0 = 16 * cb + lane % 16, 32 * kb + 8 * (lane // 16)
                assert torch.equal(img[cb, kb, lane], wb[c, k0:k0 + 8])
    imt = kernels.bf16_weight_image(w, transpose=True).view(R // 16, C // 32, 64, 8).cpu()
    # Bm = w^T: fragment (cb=2, kb=1), lane 37: column 32 + 5 of Bm = w's
    # column 37, k = 32 + 16 .. + 7 = w's rows 48 .. 55
    assert torch.equal(imt[2, 1, 37], wb[48:56, 37])


def test_grl_bf16_projections_on_own_kernels(cuda, monkeypatch):
    """configs[4]'s GatedRecurrentLayer (d = 256, L = 2048) with
    RECBLR_BF16_GEMM=1 runs all three projections' forward and input-gradient
    GEMMs on the bf16 NT kernel, the default per-shape mode (auto) four of the
    six from BF16_NT_MIN_ROWS rows on (none below), the weight gradients on
    hipBLASLt's split-K in every mode, and both agree with the hipBLASLt path
    (RECBLR_BF16_GEMM=0) to bf16 accuracy."""
    from datamining_recblr_amd.model import GatedRecurrentLayer

    calls = {"nt": 0}
    nt0 = kernels.gemm_nt_bf16

    def nt(*a, **k):
        calls["nt"] += 1
        return nt0(*a, **k)

    monkeypatch.setattr(kernels, "gemm_nt_bf16", nt)
    torch.manual_seed(5)
    layer = GatedRecurrentLayer(d_model=256).to(cuda)
    g = torch.Generator(device=cuda).manual_seed(9)
    x = torch.randn(2, 2048, 256, device=cuda, generator=g).to(BF)
    gy = torch.randn(2, 2048, 256, device=cuda, generator=g).to(BF)

    def run(on):
        prev = linear.set_bf16_gemm(on)
        try:
            layer.zero_grad(set_to_none=True)
            xx = x.clone().requires_grad_()
            y = layer(xx)
            y.backward(gy)
            return y.detach().float(), xx.grad.float(), {n: p.grad.clone() for n, p in
                                                         layer.named_parameters()}
        finally:
            linear.set_bf16_gemm(prev)

    y1, dx1, g1 = run(True)
    assert calls == {"nt": 6}, calls
    y0, dx0, g0 = run(False)
    assert calls == {"nt": 6}
    # the default per-shape mode below its row minimum (4,096 rows here):
    # every GEMM on hipBLASLt, so the results equal the "0" run bit for bit
    ys, dxs, gs = run("auto")
    assert calls == {"nt": 6}, calls
    assert torch.equal(ys, y0) and torch.equal(dxs, dx0)
    for n in g0:
        assert torch.equal(gs[n], g0[n]), n
    # ... and from the minimum on: ours for the R <= 512 NT GEMMs (in / gates
    # / out forward, out's input gradient); hipBLASLt for in.dX and gates.dX
    monkeypatch.setattr(linear, "BF16_NT_MIN_ROWS", 4096)
    ya, dxa, ga = run("auto")
    assert calls == {"nt": 10}, calls

    def rel(a, b):
        return ((a - b).abs().max() / b.abs().max()).item()

    assert rel(y1, y0) < 2e-2
    assert rel(dx1, dx0) < 2e-2
    assert rel(ya, y0) < 2e-2
    assert rel(dxa, dx0) < 2e-2
    for n in g0:
        assert rel(g1[n], g0[n]) < 2e-2, n
        assert rel(ga[n], g0[n]) < 2e-2, n


def test_bf16_linear_with_no_rows(cuda, monkeypatch):
    """An empty activation (M = 0) with the bf16 kernels selected returns an
    empty output like torch's GEMM instead of reaching the kernel's shape
    check."""
    monkeypatch.setattr(linear, "_bf16_gemm", "1")
    w = torch.randn(1024, 256, device=cuda)
    a = torch.empty(0, 256, device=cuda, dtype=BF)
    assert linear.mm_nt(a, w).shape == (0, 1024)
    dy = torch.empty(0, 1024, device=cuda, dtype=BF)
    assert linear.mm_nn(dy, w).shape == (0, 256)
