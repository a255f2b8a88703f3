"""Typed Python callers for the C-ABI entry points.

Each function validates device, dtype, shape and layout (mirroring the
reference's asserts, parallel_scan.py:86-89 and :102-104), allocates outputs
with torch's caching allocator, and launches on the current torch stream.
No function here has a CPU path: tensors must live on a ROCm GPU.
"""
from __future__ import annotations

import contextlib
import ctypes

import torch

from . import _lib
from ._lib import RB_TILE, RecBLRNativeError

__all__ = [
    "scan_fwd", "scan_bwd", "conv_silu_fwd", "conv_silu_bwd", "gate_scan_fwd",
    "gate_scan_bwd", "num_tiles", "RecBLRNativeError", "kernel_timing", "KernelTimer",
    "item_ce_fwd", "item_ce_bwd", "item_ce_probs", "item_rank", "item_scores",
    "SplitRows", "item_split_h", "item_ce_fwd_h", "item_ce_probs_h",
    "embedding_bwd", "embedding_plan",
]


class KernelTimer:
    """HIP-event timing of every C-ABI launch, recorded on the stream the
    kernel is launched on (torch's current stream).  Used by bench.py."""

    def __init__(self, only=None):
        self.only = None if only is None else frozenset(only)   # names to time (None: all)
        self.records = []   # (name, algorithmic bytes, start event, end event)
        self.detail = []    # GEMMs by shape: (label, flops, start event, end event)

    def gemm_detail(self, steps: int):
        """Per-shape GEMM times: label -> launches/step, avg us, TFLOP/s."""
        torch.cuda.synchronize()
        out = {}
        for label, flops, e0, e1 in self.detail:
            d = out.setdefault(label, {"n": 0, "ms": 0.0, "flops": 0})
            d["n"] += 1
            d["ms"] += e0.elapsed_time(e1)
            d["flops"] += flops
        return {k: {"per_step": d["n"] / steps, "avg_us": round(d["ms"] * 1e3 / d["n"], 1),
                    "tflops": round(d["flops"] / d["ms"] / 1e9, 1)}
                for k, d in sorted(out.items(), key=lambda kv: -kv[1]["ms"])}

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, nbytes, e0, e1 in self.records:
            d = out.setdefault(name, {"launches": 0, "ms": 0.0, "bytes": 0})
            d["launches"] += 1
            d["ms"] += e0.elapsed_time(e1)
            d["bytes"] += nbytes
        for d in out.values():
            d["avg_ms"] = d["ms"] / d["launches"]
            d["avg_bytes"] = d["bytes"] / d["launches"]
        return out


_timer: KernelTimer | None = None


@contextlib.contextmanager
def kernel_timing(only=None):
    """Time C-ABI launches with HIP events; `only`: the entry point names to
    time (the rest run untimed, so the timer barely perturbs the step)."""
    global _timer
    prev, _timer = _timer, KernelTimer(only)
    try:
        yield _timer
    finally:
        _timer = prev


def _launch(name: str, nbytes: int, *args, _fn: str | None = None, _flops: bool = False,
            _exp: bool = False) -> None:
    """Call C-ABI entry point `_fn or name`; timed under `name` in bench runs.
    `nbytes` is the launch's algorithmic HBM bytes, or its algorithmic FLOPs
    where `_flops` is set — exactly the names in FLOP_KERNELS (checked when
    timed, and statically by tests/test_host_logic.py)."""
    t = _timer
    call = _lib.call_exp if _exp else _lib.call
    if t is None or (t.only is not None and name not in t.only):
        call(_fn or name, *args)
        return
    if _flops != (name in FLOP_KERNELS):
        raise AssertionError(f"{name}: counted in {'FLOPs' if _flops else 'bytes'} but "
                             f"{'not ' if _flops else ''}listed in FLOP_KERNELS")
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    call(_fn or name, *args)
    e1.record()
    t.records.append((name, nbytes, e0, e1))


_tickets = {}
_lib.on_failure(_tickets.clear)


def _colsum_tickets(x: torch.Tensor, n: int) -> torch.Tensor:
    """rb_colsum_chunked's ticket counters for torch's current stream on x's
    device: zeroed once here, back at zero after every complete launch (the
    kernel's wrapping increment; calls on one stream are ordered, another
    stream gets its own).  The counters do NOT recover from a launch that did
    not complete: a stale value makes the last-arriver test fire early or
    never.  So any failed native call drops every cached counter
    (_lib.on_failure) and the next call allocates fresh zeros; a kernel that
    faults mid-launch leaves the HIP context unusable anyway (every later
    call fails, and fails loudly)."""
    key = (x.device, _stream(x))
    t = _tickets.get(key)
    if t is None or t.numel() < n:
        t = _tickets[key] = torch.zeros(max(n, 1024), device=x.device, dtype=torch.int32)
    return t


def colsum(x: torch.Tensor) -> torch.Tensor:
    """Fixed-order sum over dim -2 of a [P, C] or [M, P, C] tensor whose last
    dim is unit-stride (rb_colsum; replaces torch's sum(-2), which needs a
    semaphore memset and another launch at these shapes)."""
    _check(x, "partials")
    squeeze = x.dim() == 2
    x3 = x[None] if squeeze else x
    if x3.dim() != 3:
        raise ValueError("colsum expects [P, C] or [M, P, C]")
    if x3.stride(2) != 1:
        x3 = x3.contiguous()
    M, P, C = x3.shape
    out = torch.empty((M, C), device=x.device, dtype=torch.float32)
    if P == 0:
        return out.zero_()[0] if squeeze else out.zero_()
    rs, ms = x3.stride(1), (x3.stride(0) if M > 1 else P * x3.stride(1))
    # Few columns, many rows (per-sequence partials [B, H]): one launch would
    # have a handful of workgroups each walking thousands of rows.  Sum
    # 64-row chunks first (many workgroups), then the chunk sums — two
    # fixed-order passes, still deterministic.
    CH = 64
    if M * ((C + 63) // 64) < 64 and P >= 4 * CH and P % CH == 0 and ms == P * rs:
        # one launch (rb_colsum_chunked): chunk sums, the last arriving
        # workgroup of each column block sums them — bitwise the two passes
        nch = P // CH
        part = torch.empty((M * nch, C), device=x.device, dtype=torch.float32)
        cnt = _colsum_tickets(x, M * ((C + 63) // 64))
        _lib.call("rb_colsum_chunked", x3.data_ptr(), M, P, C, rs, CH, part.data_ptr(),
                  cnt.data_ptr(), cnt.numel(), out.data_ptr(), _stream(x))
        return out[0] if squeeze else out
    _lib.call("rb_colsum", x3.data_ptr(), M, P, C, rs, ms, out.data_ptr(), _stream(x))
    return out[0] if squeeze else out


def num_tiles(L: int) -> int:
    return (L + RB_TILE - 1) // RB_TILE


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(t: torch.Tensor) -> int:
    """hipStream_t (as int) of torch's current stream on t's device."""
    if _raw_stream is not None:
        return _raw_stream(t.device.index if t.device.index is not None
                           else torch.cuda.current_device())
    return torch.cuda.current_stream(t.device).cuda_stream


def _check(t: torch.Tensor, name: str, dtype: torch.dtype = torch.float32) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RecBLRNativeError(
            f"{name} is on {t.device}; the RecBLR HIP path needs a ROCm GPU tensor "
            "(there is no CPU fallback)")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")


ACT_DTYPES = (torch.float32, torch.bfloat16)


def _act_dtype(t: torch.Tensor, name: str) -> torch.dtype:
    """Storage dtype of the [B, L, *] activations of a recurrence kernel:
    fp32 (the reference's) or bf16 (BASELINE config 5; fp32 arithmetic)."""
    if isinstance(t, torch.Tensor) and t.dtype in ACT_DTYPES:
        return t.dtype
    _check(t, name)
    return torch.float32


def _sfx(dt: torch.dtype) -> str:
    return "_bf16" if dt == torch.bfloat16 else ""


def _row_stride(t: torch.Tensor, name: str, H: int) -> int:
    """Row stride of a [B, L, >=H] view whose (b, t) rows are uniformly spaced."""
    if t.dim() != 3 or t.shape[2] != H:
        raise ValueError(f"{name} must be [B, L, {H}], got {tuple(t.shape)}")
    B, L, _ = t.shape
    if t.stride(2) != 1 and H > 1:
        raise ValueError(f"{name} must have unit channel stride")
    rs = t.stride(1) if L > 1 else (t.stride(0) if B > 1 else H)
    if L > 1 and B > 1 and t.stride(0) != rs * L:
        raise ValueError(f"{name}: rows are not uniformly strided")
    if rs < H:
        raise ValueError(f"{name}: row stride {rs} < {H}")
    return rs


class Packed:
    """Packed variable-length sequences: sequence b occupies rows
    offsets[b] .. offsets[b+1] of a 2-D [ntok, C] activation (RecBole's
    right-padded batch without the padding; include/recblr_hip.h)."""
    __slots__ = ("offsets", "B", "L", "ntok", "pos", "last", "inv", "order", "pieces", "G",
                 "max_tiles")

    def __init__(self, offsets: torch.Tensor, L: int, ntok: int,
                 pos: torch.Tensor | None = None):
        if offsets.dtype != torch.int64 or offsets.dim() != 1 or not offsets.is_contiguous():
            raise ValueError("offsets must be a contiguous int64 [B + 1] tensor")
        if pos is not None and (pos.dtype != torch.int64 or pos.shape != (int(ntok),)
                                or not pos.is_contiguous()):
            raise ValueError("pos must be a contiguous int64 [ntok] tensor")
        self.offsets, self.B, self.L, self.ntok = offsets, offsets.numel() - 1, int(L), int(ntok)
        # optional: position of every packed row inside its sequence; lets the
        # conv forward tile the packed rows directly (rb_conv_silu_fwd_rows)
        self.pos = pos
        # optional (RecBLR._forward_packed): each batch row's last packed row
        # and its packed-sequence index; lets the last layer keep only the
        # positions gather_indexes reads (rb_gate_scan_*_last)
        self.last = None
        self.inv = None
        # optional: each packed sequence's batch row (the inverse of inv); the
        # last-position scan kernels then write / read y_last in batch order
        self.order = None
        # optional (grl_pieces): the fused GatedRecurrentLayer kernel's work
        # lists (int32 [3B + G + 1] on the device) and their count G
        self.pieces = None
        self.G = 0
        self.max_tiles = 0          # 64-row tiles of the longest work list


def _layout(t: torch.Tensor, name: str, C: int, seq: "Packed | None"):
    """(B, L, row stride, offsets pointer) of a dense [B, L, C] view or a
    packed [ntok, C] view."""
    if seq is None:
        rs = _row_stride(t, name, C)
        return t.shape[0], t.shape[1], rs, 0
    if t.dim() != 2 or t.shape != (seq.ntok, C) or (C > 1 and t.stride(1) != 1):
        raise ValueError(f"{name} must be a [{seq.ntok}, {C}] view with unit channel stride")
    rs = t.stride(0) if seq.ntok > 1 else C
    if rs < C:
        raise ValueError(f"{name}: row stride {rs} < {C}")
    if seq.offsets.device != t.device:
        raise ValueError("offsets must live on the activations' device")
    return seq.B, seq.L, rs, seq.offsets.data_ptr()


def scan_fwd(gates: torch.Tensor, tokens: torch.Tensor) -> torch.Tensor:
    dt = _act_dtype(gates, "gates")
    _check(gates, "gates", dt)
    _check(tokens, "tokens", dt)
    if gates.dim() != 3 or tokens.shape != gates.shape:
        raise ValueError("gates and tokens must both be [B, C, T] of equal shape")
    if not (gates.is_contiguous() and tokens.is_contiguous()):
        raise ValueError("gates and tokens must be contiguous")
    B, C, T = gates.shape
    states = torch.empty_like(tokens)
    if states.numel():
        _launch("rb_scan_fwd" + _sfx(dt), 3 * gates.numel() * gates.element_size(),
                gates.data_ptr(), tokens.data_ptr(), states.data_ptr(), B, C, T, _stream(gates))
    return states


def scan_bwd(gates: torch.Tensor, states: torch.Tensor, grad: torch.Tensor):
    dt = _act_dtype(gates, "gates")
    for t, n in ((gates, "gates"), (states, "states"), (grad, "grad")):
        _check(t, n, dt)
        if not t.is_contiguous():
            raise ValueError(f"{n} must be contiguous")
    if states.shape != gates.shape or grad.shape != gates.shape:
        raise ValueError("shape mismatch")
    B, C, T = gates.shape
    d_gates = torch.empty_like(gates)
    d_tokens = torch.empty_like(gates)
    if gates.numel():
        _launch("rb_scan_bwd" + _sfx(dt), 5 * gates.numel() * gates.element_size(),
                gates.data_ptr(), states.data_ptr(), grad.data_ptr(), d_gates.data_ptr(),
                d_tokens.data_ptr(), B, C, T, _stream(gates))
    return d_gates, d_tokens


def conv_silu_fwd(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor,
                  seq: Packed | None = None) -> torch.Tensor:
    """x: [B, L, H] (row-strided view ok, fp32 or bf16) or packed [ntok, H]
    with `seq`; weight: [H, K]; bias: [H] (fp32) -> xc in x's layout and dtype."""
    dt = _act_dtype(x, "x")
    _check(x, "x", dt)
    _check(weight, "conv weight")
    _check(bias, "conv bias")
    H = x.shape[-1]
    B, L, x_rs, offs = _layout(x, "x", H, seq)
    w = weight.reshape(H, -1).contiguous()
    K = w.shape[1]
    xc = torch.empty(x.shape[:-1] + (H,), device=x.device, dtype=dt)
    n = x.numel() // max(H, 1) * H
    if seq is not None and seq.pos is not None:
        if seq.pos.device != x.device:
            raise ValueError("pos must live on the activations' device")
        # packed rows tiled directly: no waves past a sequence's end
        _launch("rb_conv_silu_fwd" + _sfx(dt), 2 * n * x.element_size(), x.data_ptr(), x_rs,
                w.data_ptr(), bias.contiguous().data_ptr(), xc.data_ptr(), H, seq.ntok, H, K,
                seq.pos.data_ptr(), _stream(x), _fn="rb_conv_silu_fwd_rows" + _sfx(dt))
        return xc
    _launch("rb_conv_silu_fwd" + _sfx(dt), 2 * n * x.element_size(), x.data_ptr(), x_rs,
            w.data_ptr(), bias.contiguous().data_ptr(), xc.data_ptr(), H, B, L, H, K, offs,
            _stream(x))
    return xc


def conv_silu_bwd(x, weight, bias, g1, g2, dx, seq: Packed | None = None):
    """Writes dx (x's layout, row-strided view ok) and returns (dweight [H, K],
    dbias [H]).  g1, g2: contiguous, x's shape."""
    dt = _act_dtype(x, "x")
    _check(x, "x", dt)
    _check(g1, "g1", dt)
    _check(dx, "dx", dt)
    H = x.shape[-1]
    B, L, x_rs, offs = _layout(x, "x", H, seq)
    dx_rs = _layout(dx, "dx", H, seq)[2]
    if not g1.is_contiguous() or g1.shape != x.shape:
        raise ValueError("g1 must be contiguous, shaped like x")
    if g2 is not None:
        _check(g2, "g2", dt)
        if not g2.is_contiguous() or g2.shape != x.shape:
            raise ValueError("g2 must be contiguous, shaped like x")
    w = weight.reshape(H, -1).contiguous()
    K = w.shape[1]
    # folded partials (db_part NULL): row b = [dW[c, k] (H*K) | dbias[c] (H)],
    # one fixed-order column sum, results already in parameter layout
    part = torch.empty((B, (K + 1) * H), device=x.device, dtype=torch.float32)
    n = x.numel()
    _launch("rb_conv_silu_bwd" + _sfx(dt), (3 if g2 is None else 4) * n * x.element_size(),
            x.data_ptr(), x_rs, w.data_ptr(), bias.contiguous().data_ptr(),
            g1.data_ptr(), 0 if g2 is None else g2.data_ptr(), dx.data_ptr(), dx_rs,
            part.data_ptr(), 0, B, L, H, K, offs, _stream(x))
    sums = colsum(part)
    return sums[:H * K].view(H, K), sums[H * K:]


def gate_scan_fwd(rg, xc, z, lam, h0=None, y=None, want_carries=True, gate_b=None,
                  seq: Packed | None = None, last_only: bool = False, batch_row=None):
    """Fused alpha/beta gates + BD-LRU scan + silu(z) merge.

    rg: [B, L, 2H]; xc, z: [B, L, H] views (or packed [ntok, 2H] / [ntok, H]
    with `seq`); lam: [H]; h0: [H] (shared by every row), [B, H] (one initial
    state per row) or None; gate_b: [2H] bias added to rg inside the kernel
    (or None).  Returns (y in xc's layout, carries [B, nT, H] or None when not
    wanted).  last_only (fp32): y is only needed at each sequence's last
    position — returns y_last [B, H] instead (rb_gate_scan_fwd_last); with
    batch_row (int64 [B] permutation) sequence b's row is batch_row[b]."""
    dt = _act_dtype(xc, "xc")
    for t, n in ((rg, "rg"), (xc, "xc"), (z, "z")):
        _check(t, n, dt)
    _check(lam, "Lambda")
    H = xc.shape[-1]
    B, L, xc_rs, offs = _layout(xc, "xc", H, seq)
    rg_rs = _layout(rg, "rg", 2 * H, seq)[2]
    z_rs = _layout(z, "z", H, seq)[2]
    if seq is None and (z.shape[:2] != (B, L) or rg.shape[:2] != (B, L)):
        raise ValueError("rg, xc, z batch/length mismatch")
    if lam.shape != (H,):
        raise ValueError(f"Lambda must be [{H}]")
    h0_bs = 0
    if h0 is not None:
        _check(h0, "h0")
        if h0.shape not in ((H,), (B, H)):
            raise ValueError(f"h0 must be [{H}] or [{B}, {H}]")
        h0 = h0.contiguous()
        h0_bs = H if h0.dim() == 2 else 0
    carries = (torch.empty((B, num_tiles(L), H), device=xc.device, dtype=torch.float32)
               if want_carries else None)
    n = xc.numel()
    if last_only:
        if dt != torch.float32:
            raise ValueError("last_only is fp32")
        y_last = torch.empty((B, H), device=xc.device, dtype=dt)
        _launch("rb_gate_scan_fwd", 4 * n * 4 + B * H * 4, rg.data_ptr(), rg_rs, xc.data_ptr(),
                xc_rs, z.data_ptr(), z_rs, lam.contiguous().data_ptr(), _gb_ptr(gate_b, H),
                0 if h0 is None else h0.data_ptr(), h0_bs, y_last.data_ptr(),
                0 if carries is None else carries.data_ptr(), B, L, H, offs,
                _batch_row_ptr(batch_row, B, xc.device), _stream(xc), _fn="rb_gate_scan_fwd_last")
        return y_last, carries
    if y is None:
        y = torch.empty(xc.shape[:-1] + (H,), device=xc.device, dtype=dt)
    _check(y, "y", dt)
    y_rs = _layout(y, "y", H, seq)[2]
    _launch("rb_gate_scan_fwd" + _sfx(dt), 5 * n * xc.element_size(), rg.data_ptr(), rg_rs,
            xc.data_ptr(), xc_rs, z.data_ptr(), z_rs,
            lam.contiguous().data_ptr(), _gb_ptr(gate_b, H), 0 if h0 is None else h0.data_ptr(),
            h0_bs, y.data_ptr(), y_rs, 0 if carries is None else carries.data_ptr(), B, L, H,
            offs, _stream(xc))
    return y, carries


def _batch_row_ptr(batch_row, B, dev):
    if batch_row is None:
        return None
    if (batch_row.dtype != torch.int64 or batch_row.shape != (B,) or not batch_row.is_contiguous()
            or batch_row.device != dev):
        raise ValueError(f"batch_row must be a contiguous int64 [{B}] tensor on {dev}")
    return batch_row.data_ptr()


def _gb_ptr(gate_b, H):
    if gate_b is None:
        return None
    _check(gate_b, "gates bias")
    if gate_b.shape != (2 * H,) or not gate_b.is_contiguous():
        raise ValueError(f"gates bias must be contiguous [{2 * H}]")
    return gate_b.data_ptr()


def gate_scan_bwd(rg, xc, z, lam, carries, dy, dz, drg=None, dxc=None, dh0_rows=False,
                  gate_b=None, seq: Packed | None = None, last_only: bool = False,
                  batch_row=None):
    """Backward of gate_scan_fwd.  Writes dz (a row-strided view) and returns
    (drg, dxc, dlam [H], dgate_bias [2H], dh0), dh0 [H] (summed over rows) or
    [B, H] when dh0_rows (a per-row h0).  Layouts as in gate_scan_fwd.
    last_only: dy is [B, H], the gradient at each sequence's last position
    (zero elsewhere; rb_gate_scan_bwd_last), row batch_row[b] for sequence b
    when batch_row is given."""
    H = xc.shape[-1]
    dt = _act_dtype(xc, "xc")
    for t, n in ((rg, "rg"), (xc, "xc"), (z, "z"), (dy, "dy"), (dz, "dz")):
        _check(t, n, dt)
    _check(carries, "carries")
    B, L, xc_rs, offs = _layout(xc, "xc", H, seq)
    if last_only:
        if dt != torch.float32 or not dy.is_contiguous() or dy.shape != (B, H):
            raise ValueError(f"last_only: dy must be a contiguous fp32 [{B}, {H}]")
    elif not dy.is_contiguous() or dy.shape != xc.shape:
        raise ValueError("dy must be contiguous, shaped like xc")
    if carries.shape != (B, num_tiles(L), H) or not carries.is_contiguous():
        raise ValueError("carries shape mismatch")
    rg_rs = _layout(rg, "rg", 2 * H, seq)[2]
    z_rs = _layout(z, "z", H, seq)[2]
    dz_rs = _layout(dz, "dz", H, seq)[2]
    if drg is None:
        drg = torch.empty(xc.shape[:-1] + (2 * H,), device=xc.device, dtype=dt)
    drg_rs = _layout(drg, "drg", 2 * H, seq)[2]
    if dxc is None:
        dxc = torch.empty(xc.shape[:-1] + (H,), device=xc.device, dtype=dt)
    _check(drg, "drg", dt)
    _check(dxc, "dxc", dt)
    dxc_rs = _layout(dxc, "dxc", H, seq)[2]
    # dlam, dgate_b (2) and dh0 per-row partials in one buffer: one colsum
    part = torch.empty((4, B, H), device=xc.device, dtype=torch.float32)
    dh0_part = part[3]
    n = xc.numel()
    nbytes = (8 * n + B * H if last_only else 9 * n) * xc.element_size()
    tail = ((offs, _batch_row_ptr(batch_row, B, xc.device), _stream(xc)) if last_only
            else (offs, _stream(xc)))
    _launch("rb_gate_scan_bwd" + _sfx(dt), nbytes, rg.data_ptr(), rg_rs,
            xc.data_ptr(), xc_rs,
            z.data_ptr(), z_rs, lam.contiguous().data_ptr(), _gb_ptr(gate_b, H), carries.data_ptr(),
            dy.data_ptr(),
            drg.data_ptr(), drg_rs, dxc.data_ptr(), dxc_rs, dz.data_ptr(), dz_rs,
            part.data_ptr(), dh0_part.data_ptr(), B, L, H, *tail,
            _fn="rb_gate_scan_bwd_last" if last_only else None)
    if dh0_rows:
        sums = colsum(part[:3])
        return drg, dxc, sums[0], sums[1:].reshape(-1), dh0_part
    sums = colsum(part)
    return drg, dxc, sums[0], sums[1:3].reshape(-1), sums[3]


# ---------------------------------------------------------------- row blocks
ROW_SIZES = (16, 32, 64, 128, 256, 512, 1024)
LN_SIZES = ROW_SIZES


def _ptr(t):
    return 0 if t is None else t.data_ptr()


def _check_mask(mask, shape, name="mask"):
    if mask is None:
        return
    if mask.dtype not in (torch.uint8, torch.bool) or tuple(mask.shape) != tuple(shape):
        raise ValueError(f"{name} must be uint8/bool of shape {tuple(shape)}")
    if not mask.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _check_p(p):
    if not 0.0 <= p < 1.0:
        raise ValueError(f"dropout p must be in [0, 1), got {p}")


def row_num_parts(rows: int, width: int) -> int:
    return int(_lib.load().rb_row_num_parts(rows, width))


def add_ln_fwd(a, r, gamma, beta, eps, mask=None, seed=0, p=0.0, idx=None, save=True):
    """Fused [gather +] dropout + residual + LayerNorm over rows of d.

    a: [rows, d] (or the [V, d] table when idx [rows] is given); r: [rows, d]
    or None.  Dropout: explicit uint8 `mask` [rows, d], else Philox(`seed`)
    when p > 0.  Returns (y, s, mean, rstd); the last three are None unless
    save."""
    _check(a, "a")
    _check_p(p)
    d = a.shape[-1]
    if d not in ROW_SIZES:
        raise ValueError(f"layer norm width {d} not in {ROW_SIZES}")
    if not a.is_contiguous():
        raise ValueError("a must be contiguous")
    if idx is not None:
        if idx.dtype != torch.int64 or not idx.is_contiguous() or idx.device != a.device:
            raise ValueError("idx must be contiguous int64 on the same device")
        rows = idx.numel()
        nidx = a.shape[0]
    else:
        rows = a.numel() // d
        nidx = 0
    if r is not None:
        _check(r, "r")
        if r.numel() != rows * d or not r.is_contiguous():
            raise ValueError("r must be contiguous with rows * d elements")
    _check_mask(mask, (rows, d))
    for t, n in ((gamma, "gamma"), (beta, "beta")):
        _check(t, n)
        if t.shape != (d,) or not t.is_contiguous():
            raise ValueError(f"{n} must be contiguous [{d}]")
    dev = a.device
    y = torch.empty((rows, d), device=dev, dtype=torch.float32)
    s = mean = rstd = None
    if save:
        s = torch.empty((rows, d), device=dev, dtype=torch.float32)
        mean = torch.empty((rows,), device=dev, dtype=torch.float32)
        rstd = torch.empty((rows,), device=dev, dtype=torch.float32)
    n = rows * d
    nbytes = 4 * n * (2 + (r is not None) + (s is not None)) + (n if mask is not None else 0)
    _launch("rb_add_ln_fwd", nbytes, a.data_ptr(), _ptr(idx), nidx, _ptr(mask), int(seed),
            float(p), _ptr(r), gamma.data_ptr(), beta.data_ptr(), float(eps), y.data_ptr(),
            _ptr(s), _ptr(mean), _ptr(rstd), rows, d, _stream(a))
    return y, s, mean, rstd


def add_ln_bwd(dy, s, gamma, mean, rstd, mask=None, seed=0, p=0.0, want_ds=True,
               want_da=True, want_dbias=False, dy2=None):
    """Returns (ds, da, dgamma, dbeta, dbias); unwanted outputs are None.
    dy2: a second gradient of the same output, added on load (dy + dy2)."""
    _check(dy, "dy")
    _check_p(p)
    rows, d = s.shape
    dy = dy.reshape(rows, d)
    if not dy.is_contiguous():
        dy = dy.contiguous()
    if dy2 is not None:
        _check(dy2, "dy2")
        dy2 = dy2.reshape(rows, d)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
    _check_mask(mask, (rows, d))
    nparts = row_num_parts(rows, d)
    dev = s.device
    parts = torch.empty((3 if want_dbias else 2, nparts, d), device=dev, dtype=torch.float32)
    dgp, dbp = parts[0], parts[1]
    dbias_p = parts[2] if want_dbias else None
    ds = torch.empty((rows, d), device=dev, dtype=torch.float32) if want_ds else None
    da = torch.empty((rows, d), device=dev, dtype=torch.float32) if want_da else None
    n = rows * d
    nbytes = 4 * n * (2 + (dy2 is not None) + want_ds + want_da) + (n if mask is not None else 0)
    _launch("rb_add_ln_bwd2", nbytes, dy.data_ptr(), _ptr(dy2), s.data_ptr(), gamma.data_ptr(),
            mean.data_ptr(), rstd.data_ptr(), _ptr(mask), int(seed), float(p), _ptr(ds),
            _ptr(da), dgp.data_ptr(), dbp.data_ptr(), _ptr(dbias_p), nparts, rows, d,
            _stream(dy))
    sums = colsum(parts)
    return ds, da, sums[0], sums[1], (sums[2] if want_dbias else None)


def _rows_cols(a):
    cols = a.shape[-1]
    if cols not in ROW_SIZES:
        raise ValueError(f"row width {cols} not in {ROW_SIZES}")
    return a.numel() // cols, cols


def _bias_ptr(bias, cols):
    if bias is None:
        return None
    _check(bias, "bias")
    if bias.shape != (cols,) or not bias.is_contiguous():
        raise ValueError(f"bias must be contiguous [{cols}]")
    return bias.data_ptr()


def silu_dropout_fwd(a, mask=None, seed=0, p=0.0, bias=None):
    """u = dropout(silu(a + bias)) over rows of a (bias may be None)."""
    _check(a, "a")
    _check_p(p)
    if not a.is_contiguous():
        raise ValueError("a must be contiguous")
    rows, cols = _rows_cols(a)
    _check_mask(mask, (rows, cols))
    u = torch.empty_like(a)
    n = a.numel()
    _launch("rb_silu_dropout_fwd", 8 * n + (n if mask is not None else 0), a.data_ptr(),
            _bias_ptr(bias, cols), _ptr(mask), int(seed), float(p), u.data_ptr(), rows, cols,
            _stream(a))
    return u


def silu_dropout_bwd(a, du, mask=None, seed=0, p=0.0, want_dbias=False, bias=None):
    """Returns (da, dbias or None); bias as given to silu_dropout_fwd."""
    _check(du, "du")
    _check_p(p)
    du = du.contiguous()
    rows, cols = _rows_cols(a)
    _check_mask(mask, (rows, cols))
    da = torch.empty_like(a)
    nparts = row_num_parts(rows, cols)
    dbias_p = (torch.empty((nparts, cols), device=a.device, dtype=torch.float32)
               if want_dbias else None)
    n = a.numel()
    _launch("rb_silu_dropout_bwd", 12 * n + (n if mask is not None else 0), a.data_ptr(),
            _bias_ptr(bias, cols), _ptr(mask), int(seed), float(p), du.data_ptr(), da.data_ptr(),
            _ptr(dbias_p), nparts, rows, cols, _stream(a))
    return da, (colsum(dbias_p) if want_dbias else None)


def dropout_mask(seed, p, shape, device):
    """uint8 keep-mask of the Philox stream the row kernels use for (seed, p)."""
    _check_p(p)
    out = torch.empty(shape, dtype=torch.uint8, device=device)
    n = out.numel()
    if n % 4:
        raise ValueError("numel must be a multiple of 4")
    _launch("rb_dropout_mask", n, int(seed), float(p), out.data_ptr(), n,
            torch.cuda.current_stream(out.device).cuda_stream)
    return out


def embedding_bwd(idx, grad, num_rows, padding_idx=0, plan=None):
    """dW[v] = sum_{p: idx[p] == v} grad[p] (dW[padding_idx] = 0), deterministic.
    plan: the workspace returned by embedding_plan for the same idx (skips the
    sort), or None."""
    _check(grad, "grad")
    M = idx.numel()
    d = grad.shape[-1]
    grad = grad.reshape(M, d)
    if not grad.is_contiguous():
        grad = grad.contiguous()
    if plan is None:
        plan = embedding_plan(idx, num_rows, d)
    ws_bytes = plan.numel()
    dw = torch.empty((num_rows, d), device=grad.device, dtype=torch.float32)
    pad = -1 if padding_idx is None else int(padding_idx)
    _launch("rb_embedding_bwd", 4 * M * d + 4 * num_rows * d, grad.data_ptr(), M, d, num_rows,
            pad, dw.data_ptr(), plan.data_ptr(), ws_bytes, _stream(grad), _fn="rb_embedding_bwd_apply")
    return dw


def embedding_plan(idx, num_rows, d, stream=None):
    """Sort + segment the ids for embedding_bwd (index work only, run in the
    forward; `stream`: another stream to run on).  Returns the uint8 workspace."""
    M = idx.numel()
    if idx.dtype != torch.int64 or not idx.is_contiguous():
        raise ValueError("idx must be contiguous int64")
    if idx.device.type != "cuda":
        raise RecBLRNativeError("embedding_plan needs a GPU tensor")
    lib = _lib.load()
    ws_bytes = int(lib.rb_embedding_bwd_workspace(M, num_rows, d))
    ws = torch.empty((ws_bytes,), device=idx.device, dtype=torch.uint8)
    st = stream.cuda_stream if stream is not None else _stream(idx)
    _lib.call("rb_embedding_bwd_plan", idx.data_ptr(), M, d, num_rows, ws.data_ptr(), ws_bytes, st)
    return ws


# ---- item scoring (fp32 MFMA, no [B, V] logits) ------------------------------------
# Launches timed in FLOPs rather than bytes (bench.py reports them against the
# MFMA roofline).
FLOP_KERNELS = frozenset({"rb_item_ce_fwd", "rb_item_ce_bwd", "rb_item_ce_probs", "rb_item_rank",
                          "rb_item_scores", "rb_item_ce_fwd_h", "rb_item_ce_probs_h",
                          "rb_item_ce_probs_h_t", "rb_item_ce_probs_h_both"})


def f16_split_kernel(name: str) -> bool:
    """Kernels whose products run as three f16 MFMAs on two-part split
    operands (their FLOP peak is a third of the f16 pipe's)."""
    return name.endswith("_h") or "_h_" in name
ITEM_DIMS = (16, 32, 64, 128, 256)


def _item_operands(seq, items, target=None):
    _check(seq, "seq_output")
    _check(items, "item table")
    if seq.dim() != 2 or items.dim() != 2 or seq.shape[1] != items.shape[1]:
        raise ValueError(f"seq [B, d] and items [V, d] required, got {tuple(seq.shape)} and "
                         f"{tuple(items.shape)}")
    if seq.shape[1] not in ITEM_DIMS:
        raise ValueError(f"d = {seq.shape[1]} not in {ITEM_DIMS}")
    seq = seq.contiguous()
    items = items.contiguous()
    if target is not None:
        if target.dtype != torch.int64 or target.shape != (seq.shape[0],):
            raise ValueError("target must be int64 [B]")
        if target.device != seq.device:
            raise ValueError("target must be on the same device")
        target = target.contiguous()
    return seq, items, target


def item_ce_fwd(seq, items, target):
    """(loss, lse): mean softmax cross-entropy of seq @ items^T against target."""
    seq, items, target = _item_operands(seq, items, target)
    B, d = seq.shape
    V = items.shape[0]
    lib = _lib.load()
    ws_bytes = int(lib.rb_item_ce_workspace(B, V, d))
    ws = torch.empty((ws_bytes,), device=seq.device, dtype=torch.uint8)
    lse = torch.empty((B,), device=seq.device, dtype=torch.float32)
    loss = torch.empty((), device=seq.device, dtype=torch.float32)
    _launch("rb_item_ce_fwd", 2 * B * V * d, seq.data_ptr(), items.data_ptr(), target.data_ptr(),
            B, V, d, lse.data_ptr(), loss.data_ptr(), ws.data_ptr(), ws_bytes, _stream(seq), _flops=True)
    return loss, lse


def item_ce_bwd(seq, items, target, lse, dloss, want_seq=True, want_items=True):
    """(dseq, ditems) of item_ce_fwd for the scalar upstream gradient dloss."""
    seq, items, target = _item_operands(seq, items, target)
    _check(lse, "lse")
    _check(dloss, "dloss")
    B, d = seq.shape
    V = items.shape[0]
    dloss = dloss.reshape(1).contiguous()
    lib = _lib.load()
    ws_bytes = int(lib.rb_item_ce_workspace(B, V, d))
    ws = torch.empty((ws_bytes,), device=seq.device, dtype=torch.uint8)
    dseq = torch.empty_like(seq) if want_seq else None
    ditems = torch.empty_like(items) if want_items else None
    flops = 2 * B * V * d * (int(want_seq) + int(want_items))
    _launch("rb_item_ce_bwd", flops, seq.data_ptr(), items.data_ptr(), target.data_ptr(),
            lse.contiguous().data_ptr(), dloss.data_ptr(), B, V, d,
            dseq.data_ptr() if dseq is not None else None,
            ditems.data_ptr() if ditems is not None else None, ws.data_ptr(), ws_bytes,
            _stream(seq), _flops=True)
    return dseq, ditems


def item_ce_probs(seq, items, target, lse, dloss, item_offset=0, out=None):
    """P = (softmax - onehot) * dloss / B for the item rows `items` =
    table[item_offset : item_offset + V] ([B, V], row stride of `out`)."""
    seq, items, target = _item_operands(seq, items, target)
    _check(lse, "lse")
    _check(dloss, "dloss")
    B, d = seq.shape
    V = items.shape[0]
    if out is None:
        out = torch.empty((B, V), device=seq.device, dtype=torch.float32)
    _check(out, "probs")
    if out.shape != (B, V) or out.stride(1) != 1:
        raise ValueError("probs must be [B, V] with unit column stride")
    _launch("rb_item_ce_probs", 2 * B * V * d, seq.data_ptr(), items.data_ptr(),
            target.data_ptr(), lse.contiguous().data_ptr(), dloss.reshape(1).contiguous().data_ptr(),
            B, V, d, int(item_offset), out.data_ptr(), out.stride(0), _stream(seq), _flops=True)
    return out


class SplitRows:
    """A [n, d] fp32 matrix as the f16 pipe's two-part split image (rb_item_split_h):
    img [n, 2d] fp16 (per row d halfs x0 | d halfs x1), exps [n] int32.  Row
    slices are views (rows(v0, v1)) for the sliced CE backward."""

    __slots__ = ("img", "exps", "gmax")

    def __init__(self, img, exps, gmax=None):
        self.img, self.exps, self.gmax = img, exps, gmax

    @property
    def shape(self):
        return (self.img.shape[0], self.img.shape[1] // 2)

    def rows(self, v0, v1):
        return SplitRows(self.img[v0:v1], self.exps[v0:v1])


def item_split_h(x, group_max: bool = False) -> SplitRows:
    """x [n, d] fp32 -> SplitRows (x = 2^(e-14) (x0 + x1) per row, 22 bits);
    group_max: also .gmax [ceil(n/32)], group_absmax(x) from the same pass."""
    _check(x, "split operand")
    if x.dim() != 2 or x.shape[1] not in ITEM_DIMS:
        raise ValueError(f"[n, d] with d in {ITEM_DIMS} required, got {tuple(x.shape)}")
    x = x.contiguous()
    n, d = x.shape
    img = torch.empty((n, 2 * d), device=x.device, dtype=torch.float16)
    exps = torch.empty((n,), device=x.device, dtype=torch.int32)
    gmax = (torch.empty(((n + 31) // 32,), device=x.device, dtype=torch.float32) if group_max
            else None)
    _launch("rb_item_split_h", 8 * n * d + 4 * n, x.data_ptr(), n, d, img.data_ptr(),
            exps.data_ptr(), None if gmax is None else gmax.data_ptr(), _stream(x))
    return SplitRows(img, exps, gmax)


def _split_operands(seq, items, target):
    for sr, what in ((seq, "seq"), (items, "items")):
        if not isinstance(sr, SplitRows):
            raise TypeError(f"{what} must be a SplitRows (item_split_h)")
        if not (sr.img.is_contiguous() and sr.exps.is_contiguous()):
            raise ValueError(f"{what} split image must be contiguous")
    B, d = seq.shape
    if items.shape[1] != d or d not in ITEM_DIMS:
        raise ValueError("seq and items split images must share d in " + str(ITEM_DIMS))
    if target.dtype != torch.int64 or target.shape != (B,):
        raise ValueError("target must be int64 [B]")
    return B, items.shape[0], d, target.contiguous()


def item_ce_fwd_h(seq: SplitRows, items: SplitRows, target):
    """item_ce_fwd on split images (the f16 MFMA pipe): (loss, lse)."""
    B, V, d, target = _split_operands(seq, items, target)
    dev = seq.img.device
    lib = _lib.load()
    ws_bytes = int(lib.rb_item_ce_workspace(B, V, d))
    ws = torch.empty((ws_bytes,), device=dev, dtype=torch.uint8)
    lse = torch.empty((B,), device=dev, dtype=torch.float32)
    loss = torch.empty((), device=dev, dtype=torch.float32)
    _launch("rb_item_ce_fwd_h", 2 * B * V * d, seq.img.data_ptr(), seq.exps.data_ptr(),
            items.img.data_ptr(), items.exps.data_ptr(), target.data_ptr(), B, V, d,
            lse.data_ptr(), loss.data_ptr(), ws.data_ptr(), ws_bytes, _stream(seq.img), _flops=True)
    return loss, lse


def item_ce_probs_h(seq: SplitRows, items: SplitRows, target, lse, dloss, item_offset=0,
                    out=None):
    """item_ce_probs on split images; items = the table image's rows
    [item_offset, item_offset + V) (SplitRows.rows)."""
    B, V, d, target = _split_operands(seq, items, target)
    _check(lse, "lse")
    _check(dloss, "dloss")
    dev = seq.img.device
    if out is None:
        out = torch.empty((B, V), device=dev, dtype=torch.float32)
    _check(out, "probs")
    if out.shape != (B, V) or out.stride(1) != 1:
        raise ValueError("probs must be [B, V] with unit column stride")
    _launch("rb_item_ce_probs_h", 2 * B * V * d, seq.img.data_ptr(), seq.exps.data_ptr(),
            items.img.data_ptr(), items.exps.data_ptr(), target.data_ptr(),
            lse.contiguous().data_ptr(), dloss.reshape(1).contiguous().data_ptr(), B, V, d,
            int(item_offset), out.data_ptr(), out.stride(0), _stream(seq.img), _flops=True)
    return out


def item_ce_probs_h_t(seq: SplitRows, items: SplitRows, target, lse, dloss, item_offset=0):
    """item_ce_probs_h transposed (rb_item_ce_probs_h_t): (P^T [V, B], gmax
    [ceil(V/32)]) with gmax the max |P| of every 32-item group — the operands
    of dseq = P W (rb_gemm_tn_h) and ditems = P^T seq (rb_gemm_nt_h)."""
    B, V, d, target = _split_operands(seq, items, target)
    _check(lse, "lse")
    _check(dloss, "dloss")
    dev = seq.img.device
    ldt = (B + 3) // 4 * 4
    pt = torch.empty((V, ldt), device=dev, dtype=torch.float32)[:, :B]
    gmax = torch.zeros((V + 31) // 32, device=dev, dtype=torch.float32)
    _launch("rb_item_ce_probs_h_t", 2 * B * V * d, seq.img.data_ptr(), seq.exps.data_ptr(),
            items.img.data_ptr(), items.exps.data_ptr(), target.data_ptr(),
            lse.contiguous().data_ptr(), dloss.reshape(1).contiguous().data_ptr(), B, V, d,
            int(item_offset), pt.data_ptr(), ldt, gmax.data_ptr(), _stream(seq.img), _flops=True)
    return pt, gmax


def item_ce_probs_h_both(seq: SplitRows, items: SplitRows, target, lse, dloss, item_offset=0,
                        pad_to: int = 1):
    """Both layouts of the logits' gradient in one pass
    (rb_item_ce_probs_h_both): (P [B, Vp], P^T [V, B], bmax [ceil(B/32)],
    gmax [ceil(V/32)]) — P's columns padded with zeros to Vp = V rounded up to
    pad_to; bmax / gmax the max |P| of every 32-row / 32-item group."""
    B, V, d, target = _split_operands(seq, items, target)
    _check(lse, "lse")
    _check(dloss, "dloss")
    dev = seq.img.device
    Vp = (V + pad_to - 1) // pad_to * pad_to
    p = torch.empty((B, Vp), device=dev, dtype=torch.float32)   # pad columns zeroed in-kernel
    ldt = (B + 3) // 4 * 4
    pt = torch.empty((V, ldt), device=dev, dtype=torch.float32)[:, :B]
    maxes = torch.zeros((B + 31) // 32 + (V + 31) // 32, device=dev, dtype=torch.float32)
    bmax, gmax = maxes[:(B + 31) // 32], maxes[(B + 31) // 32:]
    _launch("rb_item_ce_probs_h_both", 2 * B * V * d, seq.img.data_ptr(), seq.exps.data_ptr(),
            items.img.data_ptr(), items.exps.data_ptr(), target.data_ptr(),
            lse.contiguous().data_ptr(), dloss.reshape(1).contiguous().data_ptr(), B, V, d,
            int(item_offset), p.data_ptr(), Vp, pt.data_ptr(), ldt, bmax.data_ptr(),
            gmax.data_ptr(), _stream(seq.img), _flops=True)
    return p, pt, bmax, gmax


def group_absmax(x: torch.Tensor) -> torch.Tensor:
    """[ceil(n/32)] max |x| over each 32-row group of a 2-D x (rb_group_absmax)."""
    _check(x, "x")
    if x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("x must be 2-D with unit column stride")
    n, c = x.shape
    out = torch.empty(((n + 31) // 32,), device=x.device, dtype=torch.float32)
    _launch("rb_group_absmax", 4 * n * c, x.data_ptr(), n, c, x.stride(0), out.data_ptr(),
            _stream(x))
    return out


def item_rank(seq, items, target, first_item=1, want_equal=True):
    """(n_greater, n_equal) int64 [B]: items in [first_item, V) other than the
    target scoring above / equal to it (-1 for an out-of-range target)."""
    seq, items, target = _item_operands(seq, items, target)
    B, d = seq.shape
    V = items.shape[0]
    lib = _lib.load()
    ws_bytes = int(lib.rb_item_rank_workspace(B, V, d))
    ws = torch.empty((ws_bytes,), device=seq.device, dtype=torch.uint8)
    gt = torch.empty((B,), device=seq.device, dtype=torch.int64)
    eq = torch.empty((B,), device=seq.device, dtype=torch.int64) if want_equal else None
    _launch("rb_item_rank", 2 * B * V * d, seq.data_ptr(), items.data_ptr(), target.data_ptr(),
            B, V, d, int(first_item), gt.data_ptr(), eq.data_ptr() if eq is not None else None,
            ws.data_ptr(), ws_bytes, _stream(seq), _flops=True)
    return gt, eq


def item_scores(seq, items):
    """scores [B, V] = seq @ items^T on the same fma chain as the CE / rank kernels."""
    seq, items, _ = _item_operands(seq, items)
    B, d = seq.shape
    V = items.shape[0]
    out = torch.empty((B, V), device=seq.device, dtype=torch.float32)
    _launch("rb_item_scores", 2 * B * V * d, seq.data_ptr(), items.data_ptr(), B, V, d,
            out.data_ptr(), _stream(seq), _flops=True)
    return out


# ---- pad-prefix state (RecBLR.py:176-179) -------------------------------------------
def _pad_args(pad_len, H, device):
    if torch.is_tensor(pad_len):
        pad = pad_len.to(device=device, dtype=torch.int64).contiguous()
        return pad, 0, pad.numel()
    return None, int(pad_len), 1


def pad_prefix_fwd(conv_b, gate_w, gate_b, lam, pad_len):
    """h0 [H] (int pad_len) or [B, H] (int64 tensor pad_len [B])."""
    for t, n in ((conv_b, "conv bias"), (gate_w, "gates weight"), (gate_b, "gates bias"),
                 (lam, "Lambda")):
        _check(t, n)
    H = lam.shape[0]
    if gate_w.shape != (2 * H, H) or conv_b.shape != (H,) or gate_b.shape != (2 * H,):
        raise ValueError("pad prefix: parameter shapes")
    pad, plen, rows = _pad_args(pad_len, H, lam.device)
    h0 = torch.empty((rows, H), device=lam.device, dtype=torch.float32)
    ws = torch.empty((5 * H,), device=lam.device, dtype=torch.float32)
    _lib.call("rb_pad_prefix_fwd", conv_b.contiguous().data_ptr(), gate_w.contiguous().data_ptr(),
              gate_b.contiguous().data_ptr(), lam.contiguous().data_ptr(),
              pad.data_ptr() if pad is not None else None, plen, rows, H, h0.data_ptr(),
              ws.data_ptr(), _stream(lam))
    return h0 if pad is not None else h0[0]


def pad_prefix_bwd(conv_b, gate_w, gate_b, lam, pad_len, dh0, into=None):
    """(dconv_b, dgate_w, dgate_b, dlam) for dh0 shaped like pad_prefix_fwd's h0.
    into = (dconv_b, dgate_w, dgate_b, dlam): add this contribution to those
    contiguous fp32 tensors in place (rb_pad_prefix_bwd accumulate) and
    return them."""
    _check(dh0, "dh0")
    H = lam.shape[0]
    pad, plen, rows = _pad_args(pad_len, H, lam.device)
    dh0 = dh0.reshape(rows, H).contiguous()
    if into is not None:
        for t, ref in zip(into, (conv_b, gate_w, gate_b, lam)):
            _check(t, "gradient")
            if t.shape != ref.shape or not t.is_contiguous():
                raise ValueError("into: contiguous tensors shaped like the parameters")
        dcb, dgw, dgb, dlam = into
    else:
        dcb = torch.empty_like(conv_b)
        dgw = torch.empty_like(gate_w)
        dgb = torch.empty_like(gate_b)
        dlam = torch.empty_like(lam)
    ws = torch.empty((5 * H,), device=lam.device, dtype=torch.float32)
    _lib.call("rb_pad_prefix_bwd", conv_b.contiguous().data_ptr(), gate_w.contiguous().data_ptr(),
              gate_b.contiguous().data_ptr(), lam.contiguous().data_ptr(),
              pad.data_ptr() if pad is not None else None, plen, rows, H, dh0.data_ptr(),
              dcb.data_ptr(), dgw.data_ptr(), dgb.data_ptr(), dlam.data_ptr(), ws.data_ptr(),
              int(into is not None), _stream(lam))
    return dcb, dgw, dgb, dlam


def pack_plan(item_seq: torch.Tensor, offsets: torch.Tensor, order: torch.Tensor, ntok: int):
    """rb_pack_plan: (ids [ntok], row_pos [ntok], inv [B], last [B]) of the
    packed layout (sequence s = batch row order[s] at rows offsets[s] ..
    offsets[s+1]); item_seq [B, L] int64 on the device."""
    for t, n in ((item_seq, "item_seq"), (offsets, "offsets"), (order, "order")):
        _check(t, n, torch.int64)
    if item_seq.dim() != 2 or item_seq.stride(1) != 1:
        item_seq = item_seq.contiguous()
    B, L = item_seq.shape
    if offsets.shape != (B + 1,) or order.shape != (B,):
        raise ValueError("offsets must be [B + 1] and order [B]")
    dev = item_seq.device
    ids = torch.empty(ntok, device=dev, dtype=torch.int64)
    pos = torch.empty(ntok, device=dev, dtype=torch.int64)
    inv = torch.empty(B, device=dev, dtype=torch.int64)
    last = torch.empty(B, device=dev, dtype=torch.int64)
    _lib.call("rb_pack_plan", item_seq.data_ptr(), item_seq.stride(0), offsets.data_ptr(),
              order.data_ptr(), B, L, ids.data_ptr(), pos.data_ptr(), inv.data_ptr(),
              last.data_ptr(), _stream(item_seq))
    return ids, pos, inv, last


class _SplitJob(ctypes.Structure):
    """rb_split_job (include/recblr_hip.h)."""
    _fields_ = [("W", ctypes.c_void_p), ("ldw", ctypes.c_int64), ("C", ctypes.c_int64),
                ("R", ctypes.c_int64), ("transpose", ctypes.c_int64), ("Wf", ctypes.c_void_p)]


MAX_SPLIT_JOBS = 32   # RB_MAX_SPLIT_JOBS


# ---- fp16 two-part split GEMMs (csrc/gemm_half.hip) --------------------------

def gemm_h_weight(w: torch.Tensor, transpose: bool = False) -> torch.Tensor:
    """f16 weight image of Bm = w (transpose=False, w [C, R]) or Bm = w^T
    (w [R, C]) for gemm_nt_h (rb_gemm_h_split_weights, one job)."""
    _check(w, "weight")
    if w.dim() != 2 or w.stride(1) != 1:
        raise ValueError("weight must be a 2-D row-major tensor")
    R, C = (w.shape[0], w.shape[1]) if transpose else (w.shape[1], w.shape[0])
    nbytes = _lib.load().rb_gemm_h_weight_bytes(C, R)
    wf = torch.empty(nbytes // 2, device=w.device, dtype=torch.float16)
    gemm_h_split_weights([(w, transpose, wf)])
    return wf


def gemm_h_split_weights(jobs) -> None:
    """(Re)build several f16 weight images in one launch
    (rb_gemm_h_split_weights): jobs = [(w, transpose, wf)]."""
    jobs = list(jobs)
    lib = _lib.load()
    for k in range(0, len(jobs), MAX_SPLIT_JOBS):
        chunk = jobs[k:k + MAX_SPLIT_JOBS]
        arr = (_SplitJob * len(chunk))()
        for d, (w, transpose, wf) in zip(arr, chunk):
            _check(w, "weight")
            if w.dim() != 2 or w.stride(1) != 1:
                raise ValueError("weight must be a 2-D row-major tensor")
            R, C = (w.shape[0], w.shape[1]) if transpose else (w.shape[1], w.shape[0])
            if wf.numel() * 2 != lib.rb_gemm_h_weight_bytes(C, R) or wf.device != w.device:
                raise ValueError("f16 weight image buffer does not match the weight")
            d.W, d.ldw, d.C, d.R = w.data_ptr(), w.stride(0), C, R
            d.transpose, d.Wf = int(transpose), wf.data_ptr()
        _lib.call("rb_gemm_h_split_weights", ctypes.addressof(arr), len(chunk),
                  _stream(chunk[0][0]))


def gemm_nt_h(a: torch.Tensor, wf: torch.Tensor, C: int, bias: torch.Tensor | None = None,
              out: torch.Tensor | None = None, rmax: torch.Tensor | None = None) -> torch.Tensor:
    """out[M, C] = a[M, R] @ Bm^T (+ bias) on the f16 pipe with Bm's f16 image
    wf (rb_gemm_nt_h); rmax [ceil(M/32)] receives max|a| per 32-row group."""
    _check(a, "a")
    if a.dim() != 2 or a.stride(1) != 1:
        raise ValueError("a must be a 2-D tensor with unit inner stride")
    M, R = a.shape
    if out is None:
        out = torch.empty((M, C), device=a.device, dtype=torch.float32)
    elif out.shape != (M, C) or out.stride(1) != 1:
        raise ValueError("out must be [M, C] with unit inner stride")
    if bias is not None:
        _check(bias, "bias")
    if rmax is not None:
        _check(rmax, "rmax")
        if rmax.numel() < (M + 31) // 32:
            raise ValueError("rmax needs ceil(M/32) entries")
    _lib.call("rb_gemm_nt_h", a.data_ptr(), a.stride(0), M, R, wf.data_ptr(), C,
              0 if bias is None else bias.data_ptr(), out.data_ptr(), out.stride(0), 0,
              0 if rmax is None else rmax.data_ptr(), _stream(a))
    return out


def gemm_nt_h_mode(mode: int = -1) -> int:
    """rb_gemm_nt_h's kernel for calls from 16,384 rows (rb_gemm_nt_h_mode):
    1 weight-stationary (csrc/gemm_ws.hip), 0 persistent tiles; -1 queries.
    Returns the previous mode."""
    return int(_lib.load().rb_gemm_nt_h_mode(int(mode)))


@contextlib.contextmanager
def nt_h_mode(mode: int):
    """Run a block with rb_gemm_nt_h_mode(mode), restoring the previous mode."""
    prev = gemm_nt_h_mode(mode)
    try:
        yield
    finally:
        gemm_nt_h_mode(prev)


def gemm_nt_h_ln_ok(a: torch.Tensor, C: int) -> bool:
    """Whether gemm_nt_h_ln takes a [M, R] operand with C outputs:
    rb_gemm_nt_h_ln's shape contract and the weight-stationary kernel selected."""
    return (a.dim() == 2 and C == 128 and a.shape[1] in (128, 256, 512) and a.stride(1) == 1
            and a.stride(0) % 4 == 0 and a.data_ptr() % 16 == 0 and gemm_nt_h_mode() == 1)


def gemm_nt_h_ln(a: torch.Tensor, wf: torch.Tensor, C: int, bias: torch.Tensor | None,
                 resid: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float,
                 seed: int, p: float, rmax: torch.Tensor | None = None):
    """(y, s, mean, rstd) of LayerNorm(dropout(a @ Bm^T + bias) + resid) from
    one GEMM epilogue (rb_gemm_nt_h_ln): add_ln_fwd(a @ Bm^T + bias, resid,
    gamma, beta, eps, seed=seed, p=p)'s outputs, s bit for bit, mean / rstd
    to fp32 rounding (RecBLR.py:142, 225-227)."""
    _check(a, "a")
    _check(resid, "resid")
    _check_p(p)
    if not gemm_nt_h_ln_ok(a, C):
        raise ValueError(f"gemm_nt_h_ln: no fused launch for {tuple(a.shape)} -> {C}")
    M, R = a.shape
    if resid.shape != (M, C) or not resid.is_contiguous():
        raise ValueError("resid must be a contiguous [M, C] tensor")
    for t, n in ((gamma, "gamma"), (beta, "beta")):
        _check(t, n)
        if t.numel() != C or t.data_ptr() % 16:
            raise ValueError(f"{n} must hold C floats, 16-byte aligned")
    if bias is not None:
        _check(bias, "bias")
    if rmax is not None:
        _check(rmax, "rmax")
        if rmax.numel() < (M + 31) // 32:
            raise ValueError("rmax needs ceil(M/32) entries")
    y = torch.empty((M, C), device=a.device, dtype=torch.float32)
    s = torch.empty_like(y)
    mean = torch.empty(M, device=a.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    _lib.call("rb_gemm_nt_h_ln", a.data_ptr(), a.stride(0), M, R, wf.data_ptr(), C,
              0 if bias is None else bias.data_ptr(), resid.data_ptr(), gamma.data_ptr(),
              beta.data_ptr(), float(eps), int(seed), float(p), y.data_ptr(), s.data_ptr(),
              mean.data_ptr(), rstd.data_ptr(), y.stride(0),
              0 if rmax is None else rmax.data_ptr(), _stream(a))
    return y, s, mean, rstd


def gemm_nt_h_act_ok(a: torch.Tensor, C: int) -> bool:
    """Whether gemm_nt_h_act takes a [M, R] operand with C outputs (freshly
    allocated contiguous outputs): rb_gemm_nt_h_act's shape contract."""
    M, R = a.shape
    return C % 256 == 0 and C <= 1024 and R % 32 == 0 and R <= 1024 and not (
        M <= 4096 and (R > 256 or C < 256))


def gemm_nt_h_act(a: torch.Tensor, wf: torch.Tensor, C: int, bias: torch.Tensor | None,
                  seed: int, p: float, rmax: torch.Tensor | None = None):
    """(out, act): out = a @ Bm^T + bias and act = dropout(silu(out)) from one
    GEMM epilogue (rb_gemm_nt_h_act) — act equals silu_dropout_fwd(out,
    seed=seed, p=p) bit for bit."""
    _check(a, "a")
    _check_p(p)
    if a.dim() != 2 or a.stride(1) != 1:
        raise ValueError("a must be a 2-D tensor with unit inner stride")
    if not gemm_nt_h_act_ok(a, C):
        raise ValueError(f"gemm_nt_h_act: no fused launch for {tuple(a.shape)} -> {C}")
    M, R = a.shape
    out = torch.empty((M, C), device=a.device, dtype=torch.float32)
    act = torch.empty_like(out)
    if bias is not None:
        _check(bias, "bias")
    if rmax is not None:
        _check(rmax, "rmax")
        if rmax.numel() < (M + 31) // 32:
            raise ValueError("rmax needs ceil(M/32) entries")
    _lib.call("rb_gemm_nt_h_act", a.data_ptr(), a.stride(0), M, R, wf.data_ptr(), C,
              0 if bias is None else bias.data_ptr(), out.data_ptr(), out.stride(0),
              0 if rmax is None else rmax.data_ptr(), act.data_ptr(), int(seed), float(p),
              _stream(a))
    return out, act


_dact_parts = None


def gemm_nt_h_dact(a: torch.Tensor, wf: torch.Tensor, C: int, pre: torch.Tensor, seed: int,
                   p: float, rmax: torch.Tensor | None = None, want_dbias: bool = True):
    """(da, dbias or None): du = a @ Bm^T never stored; da = dropout-backward
    (du) * silu'(pre) (rb_gemm_nt_h_dact) — silu_dropout_bwd(pre, du, seed=seed,
    p=p) bit for bit — and dbias = da's column sums (fixed-order partials)."""
    global _dact_parts
    _check(a, "a")
    _check(pre, "pre")
    _check_p(p)
    if a.dim() != 2 or a.stride(1) != 1:
        raise ValueError("a must be a 2-D tensor with unit inner stride")
    M, R = a.shape
    if not gemm_nt_h_act_ok(a, C) or C > 512:
        raise ValueError(f"gemm_nt_h_dact: no fused launch for {tuple(a.shape)} -> {C}")
    if pre.shape != (M, C) or not pre.is_contiguous():
        raise ValueError("pre must be a contiguous [M, C] tensor")
    if rmax is not None:
        _check(rmax, "rmax")
        if rmax.numel() < (M + 31) // 32:
            raise ValueError("rmax needs ceil(M/32) entries")
    if _dact_parts is None:
        _dact_parts = int(_lib.load().rb_gemm_nt_h_dact_parts())
    out = torch.empty((M, C), device=a.device, dtype=torch.float32)
    part = torch.empty((_dact_parts, C), device=a.device, dtype=torch.float32)
    _lib.call("rb_gemm_nt_h_dact", a.data_ptr(), a.stride(0), M, R, wf.data_ptr(), C,
              out.data_ptr(), out.stride(0), 0 if rmax is None else rmax.data_ptr(),
              pre.data_ptr(), int(seed), float(p), part.data_ptr(), _dact_parts, _stream(a))
    return out, (colsum(part) if want_dbias else None)


def gemm_tn_h(dy: torch.Tensor, x: torch.Tensor, ymax: torch.Tensor, xmax: torch.Tensor,
              splits: int) -> torch.Tensor:
    """Row-chunk partials of dW = dy^T x on the f16 pipe (rb_gemm_tn_h):
    [splits, N, K]; ymax / xmax: the 32-row-group maxima of dy / x (the
    rmax outputs of gemm_nt_h on the same operands)."""
    for t, n in ((dy, "dy"), (x, "x"), (ymax, "ymax"), (xmax, "xmax")):
        _check(t, n)
    if dy.dim() != 2 or x.dim() != 2 or dy.stride(1) != 1 or x.stride(1) != 1:
        raise ValueError("dy and x must be 2-D with unit inner stride")
    M, N = dy.shape
    K = x.shape[1]
    if x.shape[0] != M:
        raise ValueError("dy and x must have the same rows")
    if ymax.numel() < (M + 31) // 32 or xmax.numel() < (M + 31) // 32:
        raise ValueError("ymax / xmax need ceil(M/32) entries")
    parts = torch.empty((splits, N, K), device=dy.device, dtype=torch.float32)
    _lib.call("rb_gemm_tn_h", dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), M, N, K,
              ymax.data_ptr(), xmax.data_ptr(), parts.data_ptr(), splits, _stream(dy))
    return parts


def bf16_weight_image(w: torch.Tensor, transpose: bool = False) -> torch.Tensor:
    """The bf16 fragment image of Bm = w [C, R] (transpose=False) or w^T
    (transpose=True; w [R, C]) for gemm_nt_bf16 (rb_gemm_bf16_weight_image)."""
    _check(w, "w")
    if w.dim() != 2 or w.stride(1) != 1:
        raise ValueError("w must be a 2-D tensor with unit inner stride")
    C, R = (w.shape[1], w.shape[0]) if transpose else (w.shape[0], w.shape[1])
    img = torch.empty(C * R, device=w.device, dtype=torch.bfloat16)
    _lib.call("rb_gemm_bf16_weight_image", w.data_ptr(), w.stride(0), C, R, int(transpose),
              img.data_ptr(), _stream(w))
    return img


def gemm_nt_bf16(a: torch.Tensor, img: torch.Tensor, C: int,
                 bias: torch.Tensor | None = None) -> torch.Tensor:
    """out[M, C] (bf16) = a[M, R] (bf16) @ Bm^T (+ bias, fp32, added before the
    rounding) on the bf16 MFMA pipe (rb_gemm_nt_bf16); img from
    bf16_weight_image."""
    _check(a, "a", torch.bfloat16)
    _check(img, "img", torch.bfloat16)
    if a.dim() != 2 or a.stride(1) != 1:
        raise ValueError("a must be a 2-D tensor with unit inner stride")
    M, R = a.shape
    if img.numel() != C * R:
        raise ValueError("img does not match a [M, R] operand with C outputs")
    if bias is not None:
        _check(bias, "bias")
    out = torch.empty((M, C), device=a.device, dtype=torch.bfloat16)
    _lib.call("rb_gemm_nt_bf16", a.data_ptr(), a.stride(0), M, R, img.data_ptr(), C,
              0 if bias is None else bias.data_ptr(), out.data_ptr(), out.stride(0), _stream(a))
    return out


def gemm_tn_hs(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor | None = None,
               accumulate: bool = False) -> torch.Tensor:
    """dW = dy^T x [N, K] for few rows on the f16 pipe (rb_gemm_tn_hs: exact
    per-column scales, no rmax needed); with `out` and accumulate, added to it."""
    for t, n in ((dy, "dy"), (x, "x")):
        _check(t, n)
    if dy.dim() != 2 or x.dim() != 2 or dy.stride(1) != 1 or x.stride(1) != 1:
        raise ValueError("dy and x must be 2-D with unit inner stride")
    M, N = dy.shape
    K = x.shape[1]
    if x.shape[0] != M:
        raise ValueError("dy and x must have the same rows")
    if out is None:
        out = torch.empty((N, K), device=dy.device, dtype=torch.float32)
        accumulate = False
    elif out.shape != (N, K) or not out.is_contiguous() or out.dtype != torch.float32:
        raise ValueError("out must be a contiguous fp32 [N, K] tensor")
    _lib.call("rb_gemm_tn_hs", dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), M, N, K,
              out.data_ptr(), int(accumulate), _stream(dy))
    return out


def grl_pieces(lens_packed: torch.Tensor, offs: torch.Tensor, G: int) -> torch.Tensor:
    """Host-side work lists of the fused GatedRecurrentLayer kernel
    (rb_grl_fwd): whole sequences dealt to G workgroups in serpentine order
    (packed order is longest first: sequence k goes to span k % G on even
    rounds, G - 1 - k % G on odd ones), which evens the spans' row counts to
    within a fraction of a percent at the benchmark's lengths.
    lens_packed, offs: CPU int64 [B], [B + 1] in packed order.  Returns CPU
    int32 [3B + G + 1]: start row, length, packed index of each piece (in
    span order), then the G + 1 span offsets into the piece list."""
    B = lens_packed.numel()
    k = torch.arange(B)
    r, j = k // G, k % G
    span_of = torch.where(r % 2 == 0, j, G - 1 - j)
    order = torch.sort(span_of, stable=True).indices
    counts = torch.bincount(span_of, minlength=G)
    span = torch.zeros(G + 1, dtype=torch.int64)
    torch.cumsum(counts, 0, out=span[1:])
    return torch.cat([offs[:-1][order], lens_packed[order], order, span]).to(torch.int32)


def grl_max_tiles(lens_packed: torch.Tensor, G: int) -> int:
    """64-row tiles of grl_pieces' longest work list (the fused backward's
    checkpoint rows per workgroup)."""
    B = lens_packed.numel()
    k = torch.arange(B)
    r, j = k // G, k % G
    span_of = torch.where(r % 2 == 0, j, G - 1 - j)
    rows = torch.zeros(G, dtype=torch.int64).index_add_(0, span_of, lens_packed.to(torch.int64))
    return max(1, (int(rows.max()) + 63) // 64)


def grl_fwd(xz, conv_w, conv_b, wg_img, gate_b, lam, h0, seq: Packed, want_y=True,
            want_train=True, tile_carries=False):
    """The fused GatedRecurrentLayer core forward (rb_grl_fwd) on packed
    sequences: returns (y [ntok, H] or y_last [B, H] when not want_y, carries,
    xc, rg, xc_rmax) — the last four only with want_train (the three-launch
    backward's operands: 16-step carries, xc, the gates GEMM's output without
    its bias, xc's 32-row-group maxima).  tile_carries (with want_train):
    instead of those, carries = the state entering each workgroup's 64-row
    tiles [G, max_tiles, H], the only operand grl_bwd needs besides xz."""
    for t, n in ((xz, "xz"), (conv_w, "conv weight"), (conv_b, "conv bias"),
                 (gate_b, "gates bias"), (lam, "Lambda")):
        _check(t, n)
    ntok, H2 = xz.shape
    H = H2 // 2
    if seq.pieces is None or xz.stride(1) != 1 or ntok != seq.ntok:
        raise ValueError("grl_fwd needs packed sequences with their work lists")
    kc = conv_w.shape[-1]
    cw = conv_w.reshape(H, kc).contiguous()
    dev = xz.device
    y = torch.empty((ntok, H), device=dev) if want_y else None
    y_last = None if want_y else torch.empty((seq.B, H), device=dev)
    carries = xc = rg = rmax = tc = None
    nT = num_tiles(seq.L)
    if want_train and tile_carries:
        if seq.max_tiles <= 0:
            raise ValueError("tile_carries needs seq.max_tiles (grl_max_tiles)")
        tc = torch.empty((seq.G, seq.max_tiles, H), device=dev)
    elif want_train:
        carries = torch.empty((seq.B, nT, H), device=dev)
        xc = torch.empty((ntok, H), device=dev)
        rg = torch.empty((ntok, 2 * H), device=dev)
        rmax = torch.zeros((ntok + 31) // 32, device=dev)
    nbytes = (2 + (1 if want_y else 0) + (3 if xc is not None else 0)) * ntok * H * 4
    _launch("rb_grl_fwd", nbytes, xz.data_ptr(), xz.stride(0), cw.data_ptr(), kc,
            conv_b.contiguous().data_ptr(), wg_img.data_ptr(), gate_b.contiguous().data_ptr(),
            lam.contiguous().data_ptr(), 0 if h0 is None else h0.contiguous().data_ptr(),
            seq.pieces.data_ptr(), seq.B, seq.G, ntok, H,
            0 if y is None else y.data_ptr(), H, 0 if y_last is None else y_last.data_ptr(),
            0 if xc is None else xc.data_ptr(), 0 if rg is None else rg.data_ptr(),
            0 if carries is None else carries.data_ptr(), nT,
            0 if rmax is None else rmax.data_ptr(), _ptr(tc), seq.max_tiles if tc is not None else 0,
            _stream(xz), _exp=True)
    if tc is not None:
        carries = tc
    return (y if want_y else y_last), carries, xc, rg, rmax


def grl_bwd(xz, conv_w, conv_b, wg_img, wgt_img, gate_b, lam, h0, seq: Packed, tile_carries,
            dy, last_only=False, want_rmax=False):
    """Backward of grl_fwd in one launch (rb_grl_bwd) from the forward's
    tile_carries.  dy: [ntok, H], or [B, H] at each sequence's last row when
    last_only.  Returns (dxz [ntok, 2H], drg [ntok, 2H], xc [ntok, H],
    drg_rmax, xc_rmax (or None), dlam [H], dgate_b [2H], dh0 [H],
    dconv_w [H, kc], dconv_b [H])."""
    for t, n in ((xz, "xz"), (conv_w, "conv weight"), (conv_b, "conv bias"),
                 (gate_b, "gates bias"), (lam, "Lambda"), (dy, "dy")):
        _check(t, n)
    ntok, H2 = xz.shape
    H = H2 // 2
    if seq.pieces is None or xz.stride(1) != 1 or ntok != seq.ntok:
        raise ValueError("grl_bwd needs packed sequences with their work lists")
    if tile_carries.shape != (seq.G, seq.max_tiles, H) or not tile_carries.is_contiguous():
        raise ValueError("tile_carries shape mismatch")
    want = (seq.B, H) if last_only else (ntok, H)
    if tuple(dy.shape) != want or not dy.is_contiguous():
        raise ValueError(f"dy must be a contiguous fp32 {list(want)}")
    kc = conv_w.shape[-1]
    cw = conv_w.reshape(H, kc).contiguous()
    dev = xz.device
    dxz = torch.empty((ntok, H2), device=dev)
    drg = torch.empty((ntok, H2), device=dev)
    xc = torch.empty((ntok, H), device=dev)
    nr = (ntok + 31) // 32
    rmax = torch.zeros(2 * nr, device=dev) if want_rmax else None
    part = torch.empty((seq.G, 4, H), device=dev)
    cpart = torch.empty((seq.G * 8, H * kc + H), device=dev)
    nbytes = (2 + (0 if last_only else 1) + 5) * ntok * H * 4
    _launch("rb_grl_bwd", nbytes, xz.data_ptr(), xz.stride(0), cw.data_ptr(), kc,
            conv_b.contiguous().data_ptr(), wg_img.data_ptr(), wgt_img.data_ptr(),
            gate_b.contiguous().data_ptr(), lam.contiguous().data_ptr(), _ptr(h0),
            seq.pieces.data_ptr(), seq.B, seq.G, ntok, H, tile_carries.data_ptr(), seq.max_tiles,
            0 if last_only else dy.data_ptr(), dy.data_ptr() if last_only else 0,
            dxz.data_ptr(), H2, drg.data_ptr(), xc.data_ptr(),
            0 if rmax is None else rmax.data_ptr(), 0 if rmax is None else rmax[nr:].data_ptr(),
            part.data_ptr(), cpart.data_ptr(), _stream(xz), _exp=True)
    sums = colsum(part.view(seq.G, 4 * H)).view(4, H)
    csum = colsum(cpart)
    return (dxz, drg, xc, None if rmax is None else rmax[:nr], None if rmax is None else rmax[nr:],
            sums[0], sums[1:3].reshape(-1), sums[3], csum[:H * kc].view(H, kc), csum[H * kc:])
