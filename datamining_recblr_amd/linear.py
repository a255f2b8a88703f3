"""Projection GEMMs with split-K weight gradients.

Every projection of the encoder is tall and skinny: X [B*L, K] @ W^T with
B*L = 409,600 rows at the benchmark shape and K, N in {128, 256, 512}.  The
forward and dX GEMMs have plenty of output tiles, but the weight gradient
dW = dY^T X [N, K] has only a few dozen tiles and a 409,600-long reduction, on
which the BLAS picks un-split kernels running at ~46 TFLOP/s (MI355X fp32
MFMA peak 157).  Splitting the reduction into S row blocks as one batched GEMM
([S, N, M/S] x [S, M/S, K], ~1000 tiles) and summing the S partials in a fixed
order runs 2-4.5x faster (tools/gemm_probe.py) and is deterministic.

The forward and input-gradient GEMMs of the packed [ntok, *] projections run
on split-operand MFMA kernels (``mm_nt`` / ``mm_nn``), selected by
RECBLR_GEMM:
  f16x3  (default, csrc/gemm_half.hip): every fp32 operand scaled by an exact
         power of two and split into two fp16 parts, three products, fp32
         accumulation — error vs fp64 at or below hipBLASLt's fp32 kernels;
  torch  (or RECBLR_SPLIT_GEMM=0): hipBLASLt/rocBLAS fp32 through torch.
(Round 1's bf16x6 kernel — three exact bf16 parts, six products — was kept
for A/B until round 4 and is in git history.)
Their speed does not depend on the row count, which changes every batch once
the sequences are packed (RecBLR._forward_packed): there hipBLASLt's untuned
heuristic picks run at 86-117 TFLOP/s.  Shapes they do not
cover (and small M) stay on torch.  The math is exactly nn.Linear's
(RecBLR.py:162,165,167,213,214).  The input-gradient GEMM never accumulates
into a residual gradient: the consumer of that gradient adds it while loading
(rb_add_ln_bwd2's dy2, rb_conv_silu_bwd's g2; see blocks.ResidualGrad).
"""
from __future__ import annotations

import os
import weakref

import torch

from . import _lib, gemm_tuning, kernels

__all__ = ["linear", "wgrad", "LinearFn", "mm_nt", "mm_nn", "split_gemm_enabled",
           "HipLinearForward", "has_hooks", "fire_hooks"]

_GEMM = os.environ.get("RECBLR_GEMM", "f16x3")
if _GEMM not in ("f16x3", "torch"):
    raise ValueError(f"RECBLR_GEMM must be f16x3 or torch, got {_GEMM!r}")
_split_on = os.environ.get("RECBLR_SPLIT_GEMM", "1") != "0" and _GEMM != "torch"
_half = _GEMM == "f16x3"
# weight gradients on the f16 pipe (rb_gemm_tn_h) when both operands' row-group
# maxima are known (RECBLR_TN=0: hipBLASLt split-K, below)
_tn_on = os.environ.get("RECBLR_TN", "1") != "0"
_cache_on = os.environ.get("RECBLR_SPLIT_CACHE", "1") != "0"
# few-rows weight gradients on rb_gemm_tn_hs (RECBLR_SMALL_TN=1); off by
# default: at B = 2048 rows it measured 59 us against hipBLASLt's 18 us
# (profiles/r03_v1_bench.log: 32-64 workgroups of column-strided loads)
_small_tn = os.environ.get("RECBLR_SMALL_TN", "0") == "1"

# Split images of the weights, kept across calls: (id(w), transpose) ->
# [weakref(w), data_ptr, (version, optimizer steps), wf].  An entry is current
# while the weight's storage, its version counter (every in-place update:
# optimizer steps, load_state_dict, nn.init) and the count of optimizer steps
# taken anywhere (torch.optim step hook: also covers optimizers that write
# through .data) are unchanged; the first stale lookup of a training step
# refreshes every stale entry of that device in one launch
# (rb_gemm_h_split_weights) instead of one launch per GEMM call.  Code that
# rewrites weights through .data outside torch.optim calls
# invalidate_split_cache() (or sets RECBLR_SPLIT_CACHE=0).
_split_cache: dict = {}
_opt_steps = [0]
# RECBLR_SPLIT_CACHE_CHECK=1: every cached image is compared with a fresh
# split of the weight at each use and a stale one raises (debug mode for code
# that rewrites weights behind torch.optim's back, e.g. through .data)
_cache_check = os.environ.get("RECBLR_SPLIT_CACHE_CHECK", "0") == "1"


class StaleSplitCacheError(RuntimeError):
    """A cached split weight image no longer matches its weight."""


def _count_step(*_args, **_kw):
    _opt_steps[0] += 1


try:
    from torch.optim.optimizer import register_optimizer_step_post_hook
except ImportError:   # older torch: version counters only
    register_optimizer_step_post_hook = None
if register_optimizer_step_post_hook is not None:
    register_optimizer_step_post_hook(_count_step)


def invalidate_split_cache() -> None:
    _split_cache.clear()
    _bf16_cache.clear()


def _stamp(w: torch.Tensor):
    return (w._version, _opt_steps[0])


def _make_image(w, transpose):
    return kernels.gemm_h_weight(w, transpose=transpose)


def _weight_split(w: torch.Tensor, transpose: bool) -> torch.Tensor:
    """The f16 weight image of w (transpose: of w^T), cached."""
    if not _cache_on:
        return _make_image(w, transpose)
    key = (id(w), transpose)
    e = _split_cache.get(key)
    if e is not None and e[0]() is w and e[1] == w.data_ptr() and e[2] == _stamp(w):
        if _cache_check and not torch.equal(e[3], _make_image(w, transpose)):
            raise StaleSplitCacheError(
                "cached split image of a weight is stale: the weight was rewritten without "
                "a torch.optim step or a version bump; call linear.invalidate_split_cache()")
        return e[3]
    if e is None or e[0]() is not w or e[1] != w.data_ptr():
        # new (or re-allocated) weight: its own split, then cached
        wf = _make_image(w, transpose)
        _split_cache[key] = [weakref.ref(w), w.data_ptr(), _stamp(w), wf]
        return wf
    # stale after an in-place update: refresh all stale entries at once
    jobs, fresh = [], []
    for k, ent in list(_split_cache.items()):
        ww = ent[0]()
        if ww is None or ww.data_ptr() != ent[1]:
            del _split_cache[k]
            continue
        if _stamp(ww) != ent[2] and ww.device == w.device:
            jobs.append((ww, k[1], ent[3]))
            fresh.append(ent)
    kernels.gemm_h_split_weights(jobs)
    for ent in fresh:
        ent[2] = _stamp(ent[0]())
    return e[3]


def split_gemm_enabled() -> bool:
    return _split_on


# f16x3: any row count (below one persistent round, and for the rows past the
# last whole round, rb_gemm_nt_h runs its few-rows kernel, csrc/gemm_small.hip)
HALF_MIN_ROWS = 1


def _split_ok(a: torch.Tensor, C: int, R: int) -> bool:
    return (_split_on and _half and a.is_cuda and a.dim() == 2 and a.shape[0] >= HALF_MIN_ROWS
            and C % 32 == 0 and R % 32 == 0 and a.stride(1) == 1 and a.stride(0) % 4 == 0
            and a.data_ptr() % 16 == 0 and a.dtype == torch.float32 and C <= 1024)


def gemm_format() -> str:
    """The split GEMM format in use: 'f16x3' or 'torch'."""
    return _GEMM if _split_on else "torch"


# rb_gemm_nt_h's kernel for its large calls (>= 16,384 rows): the weight-
# stationary kernel (csrc/gemm_ws.hip, round 6: the weight slice resident in
# registers, A streamed once per column tile, exact row scales) or, with
# RECBLR_NT_WS=0, round 5's persistent 256-row tiles (csrc/gemm_half.hip).
_NT_WS = os.environ.get("RECBLR_NT_WS", "1")
if _NT_WS not in ("0", "1"):
    raise ValueError(f"RECBLR_NT_WS must be 0 or 1, got {_NT_WS!r}")
_nt_ws_applied = None


def _apply_nt_ws() -> None:
    global _nt_ws_applied
    if _nt_ws_applied != _NT_WS:
        _lib.load().rb_gemm_nt_h_mode(int(_NT_WS))
        _nt_ws_applied = _NT_WS


def set_nt_ws(on: bool) -> bool:
    """Select the weight-stationary NT kernel (True) or the persistent tiles
    (False) for rb_gemm_nt_h's large calls (bench A/B); returns the previous
    setting."""
    global _NT_WS
    prev = _NT_WS == "1"
    _NT_WS = "1" if on else "0"
    _apply_nt_ws()
    return prev


def rmax_wanted() -> bool:
    """Whether weight gradients take the f16 pipe's row-group maxima (rmax)."""
    return _half and _tn_on and _split_on


def rmax_buffer(a: torch.Tensor, C: int, R: int) -> torch.Tensor | None:
    """A [ceil(M/32)] buffer for the row-group maxima of `a` that the f16 GEMM
    writes (the weight-gradient kernel's operand scale) — None when a's GEMM
    with C outputs and R inputs will not run on the f16 kernel."""
    if _half and _tn_on and _split_ok(a, C, R):
        return torch.empty((a.shape[0] + 31) // 32, device=a.device, dtype=torch.float32)
    return None


# bf16 activations (BASELINE configs[4]): the projections on our bf16 MFMA
# kernels (csrc/gemm_bf16.hip) or torch's bf16 GEMMs (hipBLASLt), per shape.
# RECBLR_BF16_GEMM:
#   "auto" (default) — ours where they measured faster at configs[4]: the
#     NT kernel for R <= 512 inputs (the three forward GEMMs and out's input
#     gradient: 4-9% faster than hipBLASLt, profiles/r05_bfmid_shapes.txt);
#     hipBLASLt for the K = 1024 input gradients of the in / gates
#     projections (7-14% faster there);
#   "1" — ours on every NT shape; "0" — hipBLASLt on every shape.
# The weight gradients of bf16 activations always run on torch's batched
# split-K + rb_colsum (round 5's rb_gemm_tn_bf16 measured 4-24% behind it,
# profiles/r05_tn48_shapes.txt, and was removed in round 6).
# The weight's bf16 fragment images (W for the forward, W^T for the input
# gradient) are cached per weight version like the split images.
BF16_NT_MAX_R = 512
# auto: our NT kernel only from one persistent round of 256-row tiles per CU
# (256 CUs x 256 rows): it was measured against hipBLASLt only at configs[4]'s
# 2,097,152 rows, and below a round the persistent grid runs partly empty —
# smaller bf16 GEMMs stay on hipBLASLt ("1" forces ours at any size)
BF16_NT_MIN_ROWS = 65536
_BF16_MODES = ("auto", "1", "0")
_bf16_gemm = os.environ.get("RECBLR_BF16_GEMM", "auto")
if _bf16_gemm not in _BF16_MODES:
    raise ValueError(f"RECBLR_BF16_GEMM must be one of {_BF16_MODES}, got {_bf16_gemm!r}")
_bf16_cache: dict = {}


def set_bf16_gemm(mode) -> str:
    """Switch the bf16 projection kernels (A/B in bench.py): "auto", "1"
    (True) or "0" (False); returns the previous mode."""
    global _bf16_gemm
    m = {True: "1", False: "0"}.get(mode, mode) if isinstance(mode, bool) else str(mode)
    if m not in _BF16_MODES:
        raise ValueError(f"bf16 GEMM mode must be one of {_BF16_MODES}, got {mode!r}")
    prev, _bf16_gemm = _bf16_gemm, m
    return prev


def _bf16_image(w: torch.Tensor, transpose: bool) -> torch.Tensor:
    key = (id(w), transpose)
    e = _bf16_cache.get(key)
    if (_cache_on and e is not None and e[0]() is w and e[1] == w.data_ptr()
            and e[2] == _stamp(w)):
        return e[3]
    img = kernels.bf16_weight_image(w, transpose)
    if _cache_on:
        for k in [k for k, v in _bf16_cache.items() if v[0]() is None]:
            del _bf16_cache[k]
        _bf16_cache[key] = (weakref.ref(w), w.data_ptr(), _stamp(w), img)
    return img


def _bf16_ok(a: torch.Tensor, w: torch.Tensor, C: int, R: int) -> bool:
    return (_bf16_gemm != "0"
            and (_bf16_gemm == "1" or (R <= BF16_NT_MAX_R and a.shape[0] >= BF16_NT_MIN_ROWS))
            and a.dtype == torch.bfloat16 and w.dtype == torch.float32 and a.is_cuda
            and a.dim() == 2 and a.shape[0] > 0 and a.stride(1) == 1 and a.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and w.stride(1) == 1 and R % 64 == 0 and C % 256 == 0)


def mm_nt(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None,
          rmax: torch.Tensor | None = None) -> torch.Tensor:
    """a [M, K] @ w[N, K]^T (+ bias): F.linear's forward GEMM.  bf16
    activations (config 5) use the weight rounded to bf16 (bf16 MFMA, fp32
    accumulation, bf16 output).  rmax: from rmax_buffer(a, N, K)."""
    if a.dtype != w.dtype and _bf16_ok(a, w, w.shape[0], w.shape[1]):
        b = None if bias is None else bias.contiguous()
        return kernels.gemm_nt_bf16(a, _bf16_image(w, False), w.shape[0], bias=b)
    if a.dtype != w.dtype:
        wb = w.to(a.dtype)
        return torch.addmm(bias.to(a.dtype), a, wb.t()) if bias is not None else a @ wb.t()
    N, K = w.shape
    if _split_ok(a, N, K):
        _apply_nt_ws()
        return kernels.gemm_nt_h(a, _weight_split(w, False), N, bias=bias, rmax=rmax)
    return torch.addmm(bias, a, w.t()) if bias is not None else torch.mm(a, w.t())


# The FeedForward's first projection with dropout(silu(.)) in its epilogue
# (rb_gemm_nt_h_act): the activation kernel's re-read of the GEMM output is
# gone.  RECBLR_FFN_ACT=0: the GEMM and rb_silu_dropout_fwd as two launches.
_act_fused = os.environ.get("RECBLR_FFN_ACT", "1") != "0"
# below one persistent round (the gathered last-layer tail, B = 2,048 rows)
# the fused launches run on a few dozen workgroups and measured slower than
# the two launches (mm_nn_dact 30.7 us at 2,048 rows; profiles/r03_ffnact_bench.log)
ACT_MIN_ROWS = 16384


def set_ffn_act_fused(on: bool) -> bool:
    """Switch the fused FeedForward activation (A/B in bench.py); returns the
    previous setting."""
    global _act_fused
    prev, _act_fused = _act_fused, bool(on)
    return prev


def mm_nt_act_ok(a: torch.Tensor, w: torch.Tensor) -> bool:
    """Whether mm_nt_act applies to a [M, K] @ w [N, K]^T (else: the GEMM and
    the activation kernel as two launches)."""
    N, K = w.shape
    return (_act_fused and _half and a.dtype == w.dtype and a.shape[0] >= ACT_MIN_ROWS
            and _split_ok(a, N, K) and kernels.gemm_nt_h_act_ok(a, N))


def mm_nt_act(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None, seed: int, p: float,
              rmax: torch.Tensor | None = None):
    """(a @ w^T + bias, dropout(silu(a @ w^T + bias))) from one f16x3 GEMM
    launch (where mm_nt_act_ok)."""
    return kernels.gemm_nt_h_act(a, _weight_split(w, False), w.shape[0], bias, seed, p, rmax=rmax)


# The residual + dropout + LayerNorm after a projection to d = 128 in the
# GEMM's epilogue (rb_gemm_nt_h_ln; the FeedForward's w_2 and the recurrent
# layer's out-projection): the LayerNorm kernel's re-read of the GEMM output
# and the output's write are gone.  RECBLR_LN_EPI=0: the GEMM and
# rb_add_ln_fwd as two launches.
_ln_fused = os.environ.get("RECBLR_LN_EPI", "1") != "0"
if os.environ.get("RECBLR_LN_EPI", "1") not in ("0", "1"):
    raise ValueError("RECBLR_LN_EPI must be 0 or 1")


def set_ln_fused(on: bool) -> bool:
    """Switch the LayerNorm GEMM epilogue (A/B in bench.py); returns the
    previous setting."""
    global _ln_fused
    prev, _ln_fused = _ln_fused, bool(on)
    return prev


def mm_nt_ln_ok(a: torch.Tensor, w: torch.Tensor) -> bool:
    """Whether mm_nt_ln applies to a [M, K] @ w [N, K]^T (N = 128; else the
    GEMM and rb_add_ln_fwd as two launches)."""
    N, K = w.shape
    if not (_ln_fused and _half and a.dtype == w.dtype and a.shape[0] >= ACT_MIN_ROWS
            and _split_ok(a, N, K)):
        return False
    _apply_nt_ws()
    return kernels.gemm_nt_h_ln_ok(a, N)


def mm_nt_ln(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None, resid: torch.Tensor,
             gamma: torch.Tensor, beta: torch.Tensor, eps: float, seed: int, p: float,
             rmax: torch.Tensor | None = None):
    """(y, s, mean, rstd) = LayerNorm(dropout(a @ w^T + bias) + resid) and its
    saved statistics from one f16x3 GEMM launch (where mm_nt_ln_ok)."""
    return kernels.gemm_nt_h_ln(a, _weight_split(w, False), w.shape[0], bias, resid, gamma, beta,
                                eps, seed, p, rmax=rmax)


def mm_nn_dact_ok(dy: torch.Tensor, w: torch.Tensor) -> bool:
    """Whether mm_nn_dact applies to dy [M, N] @ w [N, K]."""
    N, K = w.shape
    return (_act_fused and _half and dy.dtype == w.dtype and K <= 512
            and dy.shape[0] >= ACT_MIN_ROWS and _split_ok(dy, K, N)
            and kernels.gemm_nt_h_act_ok(dy, K))


def mm_nn_dact(dy: torch.Tensor, w: torch.Tensor, pre: torch.Tensor, seed: int, p: float,
               rmax: torch.Tensor | None = None):
    """(da, dbias): the activation backward of mm_nt_act's act fused into the
    input-gradient GEMM du = dy @ w (du never stored; where mm_nn_dact_ok)."""
    return kernels.gemm_nt_h_dact(dy, _weight_split(w, True), w.shape[1], pre, seed, p,
                                  rmax=rmax)


def mm_nn(dy: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None,
          rmax: torch.Tensor | None = None) -> torch.Tensor:
    """dy [M, N] @ w [N, K] (the input gradient of F.linear); with `out`,
    accumulated into it in place (out += dy @ w)."""
    if dy.dtype != w.dtype and out is None and _bf16_ok(dy, w, w.shape[1], w.shape[0]):
        return kernels.gemm_nt_bf16(dy, _bf16_image(w, True), w.shape[1])
    if dy.dtype != w.dtype:
        wb = w.to(dy.dtype)
        return out.addmm_(dy, wb) if out is not None else dy @ wb
    N, K = w.shape
    if _split_ok(dy, K, N):
        _apply_nt_ws()
        r = kernels.gemm_nt_h(dy, _weight_split(w, True), K, rmax=rmax)
        return r if out is None else out.add_(r)
    if out is not None:
        return out.addmm_(dy, w)
    return torch.mm(dy, w)


SPLIT_K = 64
MIN_ROWS_FOR_SPLIT = 16384
# few-thousand-row weight gradients (the gathered last-layer tail, B rows)
# with both operands' row-group maxima known: rb_gemm_tn_h with one 32-row
# group per split (S = M / 32 <= 64) plus the column sum; at B = 2,048 the
# three tail shapes take 16-22 us each, 55.6 us together against hipBLASLt's
# 56.4 us (profiles/r03_ceb_bench_tnfew.log, r03_tnfew_bench.log: 19-22 us on
# another lease) — the step then runs no library GEMM (RECBLR_TN_FEW=0:
# hipBLASLt)
TN_FEW_MIN_ROWS = 2048
_tn_few = os.environ.get("RECBLR_TN_FEW", "1") != "0"


_ncus = {}


def _tn_splits(dev, nt: int) -> int:
    n = _ncus.get(dev)
    if n is None:
        n = _ncus[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
    return max(8, (2 * n // nt) // 8 * 8)   # ~2 workgroups per CU, a multiple of 8


def wgrad(dy2: torch.Tensor, x2: torch.Tensor, splits: int = SPLIT_K,
          ymax: torch.Tensor | None = None, xmax: torch.Tensor | None = None) -> torch.Tensor:
    """dW = dy2^T @ x2 for dy2 [M, N], x2 [M, K] (row-strided views allowed).
    With both operands' row-group maxima (ymax, xmax: the rmax outputs of the
    f16 GEMMs that read dy2 and x2), on the f16 pipe (rb_gemm_tn_h: fixed-order
    row-chunk partials); else hipBLASLt's batched split-K (bf16 activations,
    config 5: bf16 partials, summed in fp32; the result is fp32 like the
    parameter)."""
    M = dy2.shape[0]
    N, K = dy2.shape[1], x2.shape[1]
    if (ymax is not None and xmax is not None
            and (M >= MIN_ROWS_FOR_SPLIT or (_tn_few and M >= TN_FEW_MIN_ROWS))
            and N % 128 == 0
            and K % 128 == 0 and dy2.stride(1) == 1 and x2.stride(1) == 1
            and dy2.stride(0) % 4 == 0 and x2.stride(0) % 4 == 0
            and dy2.data_ptr() % 16 == 0 and x2.data_ptr() % 16 == 0):
        S = _tn_splits(dy2.device, (N // 128) * (K // 128))
        if M < MIN_ROWS_FOR_SPLIT:   # at least one 32-row group per split
            S = max(8, min(S, M // 32 // 8 * 8))
        parts = kernels.gemm_tn_h(dy2, x2, ymax, xmax, S)
        return kernels.colsum(parts.view(S, -1)).view(N, K)
    if (_small_tn and _half and _split_on and _tn_on and M < MIN_ROWS_FOR_SPLIT and N % 32 == 0
            and K % 32 == 0 and dy2.dtype == torch.float32 and x2.dtype == torch.float32
            and dy2.is_cuda and dy2.stride(1) == 1 and x2.stride(1) == 1):
        # few rows (the gathered last-layer tail): exact per-column scales
        return kernels.gemm_tn_hs(dy2, x2)
    if M < MIN_ROWS_FOR_SPLIT or splits <= 1:
        return (dy2.t() @ x2).float()
    mk = M // splits
    main = mk * splits
    a = dy2[:main].unflatten(0, (splits, mk)).transpose(1, 2)
    b = x2[:main].unflatten(0, (splits, mk))
    # the M % splits leftover rows (packed batches have any M) go to one more
    # partial slot, summed by the same fixed-order colsum (no extra add pass)
    parts = torch.empty((splits + (main < M), N, K), device=dy2.device, dtype=dy2.dtype)
    torch.bmm(a, b, out=parts[:splits])
    if main < M:
        torch.mm(dy2[main:].t(), x2[main:], out=parts[splits])
    if parts.dtype != torch.float32:
        parts = parts.float()
    return kernels.colsum(parts.view(parts.shape[0], -1)).view(N, K)


def _label(fn, args) -> str:
    """GEMM label for the bench's per-shape breakdown: op[M x K -> N]."""
    name = getattr(fn, "__name__", "gemm")
    if name in ("mm_nt", "mm_nn", "mm_nt_act", "mm_nn_dact") and len(args) >= 2:
        a, w = args[0], args[1]
        n_out = w.shape[1] if name.startswith("mm_nn") else w.shape[0]
        return f"{name}[{a.shape[0]}x{a.shape[1]}->{n_out}]"
    if name == "wgrad" and len(args) >= 2:
        return f"wgrad[{args[0].shape[0]}:{args[0].shape[1]}x{args[1].shape[1]}]"
    return name


def _timed(kind, flops, fn, *args, **kw):
    """Run a GEMM, bracketed by HIP events when bench.py's kernel timer is on."""
    t = kernels._timer
    if t is None or t.only is not None:
        return fn(*args, **kw)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    out = fn(*args, **kw)
    e1.record()
    t.records.append((kind, flops, e0, e1))
    t.detail.append((_label(fn, args), flops, e0, e1))
    return out


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, slot=None):
        x2 = x.reshape(-1, x.shape[-1])
        flops = 2 * x2.shape[0] * x2.shape[1] * weight.shape[0]
        rx = rmax_buffer(x2, weight.shape[0], weight.shape[1]) if ctx.needs_input_grad[1] else None
        y = _timed("gemm", flops, mm_nt, x2, weight, bias, rmax=rx)
        ctx.rx = rx
        ctx.save_for_backward(x2, weight)
        ctx.has_bias = bias is not None
        ctx.slot = slot
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        flops = 2 * x2.shape[0] * x2.shape[1] * weight.shape[0]
        dx = dw = db = None
        ry = None
        if ctx.needs_input_grad[0]:
            slot = ctx.slot
            ry = rmax_buffer(dy2, weight.shape[1], weight.shape[0]) if ctx.rx is not None else None
            dx = _timed("gemm", flops, mm_nn, dy2, weight, rmax=ry)
            if slot is not None and slot.ds is not None:
                if slot.rows is not None:        # residual of gathered rows
                    dx.index_add_(0, slot.rows, slot.ds.view(-1, weight.shape[1]))
                    slot.ds = None
                elif not slot.taken:             # nobody downstream adds it
                    dx.add_(slot.ds.view(-1, weight.shape[1]))
                    slot.ds = None
                # else: x's producer adds slot.ds while loading (rb_add_ln_bwd2)
            dx = dx.view(*dy.shape[:-1], weight.shape[1])
        if ctx.needs_input_grad[1]:
            dw = _timed("gemm", flops, wgrad, dy2, x2, ymax=ry, xmax=ctx.rx)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = (kernels.colsum(dy2.contiguous()) if dy2.dtype == torch.float32
                  else dy2.sum(0, dtype=torch.float32))
        return dx, dw, db, None


def has_hooks(module: torch.nn.Module) -> bool:
    """Forward (pre-)hooks registered on `module` or globally."""
    g = torch.nn.modules.module
    return bool(module._forward_hooks or module._forward_pre_hooks
                or g._global_forward_hooks or g._global_forward_pre_hooks)


def fire_hooks(module: torch.nn.Module, args: tuple, output) -> None:
    """Run the forward pre-hooks and hooks nn.Module.__call__ would run for
    `module(*args) -> output`, for a module whose arithmetic happens inside a
    fused kernel (the gates Linear inside the BD-LRU kernels, the FeedForward
    Linears): observers — FLOP counters such as RecBole's get_flops
    (run.py:76-77), profilers — see the call.  A hook that returns a value
    (would replace the input or the output) cannot be honoured there and
    raises."""
    g = torch.nn.modules.module
    for hook in (*g._global_forward_pre_hooks.values(), *module._forward_pre_hooks.values()):
        if hook(module, args) is not None:
            raise NotImplementedError(
                "a forward pre-hook that modifies the input of a Linear fused into a RecBLR "
                "HIP kernel is not supported")
    for hook in (*g._global_forward_hooks.values(), *module._forward_hooks.values()):
        if hook(module, args, output) is not None:
            raise NotImplementedError(
                "a forward hook that replaces the output of a Linear fused into a RecBLR "
                "HIP kernel is not supported")


class HipLinearForward:
    """nn.Linear.forward on the HIP path, installed per instance
    (``m.forward = HipLinearForward(m)``) so the module's own __call__ —
    hooks included — runs it while its type stays nn.Linear (FLOP counters
    dispatch on the exact type).  A residual-gradient slot for the next call
    is passed through the ``_recblr_slot`` attribute (blocks.ResidualGrad).
    A plain object (not a bound method) so the module still pickles."""

    def __init__(self, module: torch.nn.Linear):
        self.module = module

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        m = self.module
        slot = m.__dict__.get("_recblr_slot")
        m.__dict__["_recblr_slot"] = None
        return linear(x, m, slot)


def linear(x: torch.Tensor, module: torch.nn.Linear, slot=None) -> torch.Tensor:
    """module(x) with the split-K weight gradient; `slot` (blocks.ResidualGrad)
    adds a residual gradient inside the dX GEMM."""
    if _tuned is None and x.is_cuda:
        _load_tuned()
    return LinearFn.apply(x, module.weight, module.bias, slot)


_tuned = None


def _load_tuned():
    global _tuned
    _tuned = gemm_tuning.use_tuned_gemms()
