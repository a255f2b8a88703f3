"""Adam on the native library (rb_adam_step): the training step's optimizer
update over every parameter in one launch.

torch.optim.Adam semantics (L2 weight_decay, no amsgrad / maximize) — the
optimizer RecBole's Trainer builds for RecBLR (run.py, learner 'adam').
torch's fused Adam walks its tensor lists in 64K-element chunks, one
workgroup each, so the encoder's ~2.1 M parameters occupy a few dozen of 256
CUs (48 us per step, profiles/r03_v12_kernel_stats.csv); csrc/adam.hip
spreads every tensor over the chip.  State per parameter: exp_avg,
exp_avg_sq and step (torch's names, so state_dict() reads alike).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib, kernels

MAX_ADAM_JOBS = 48   # RB_MAX_ADAM_JOBS


class _AdamJob(ctypes.Structure):
    """rb_adam_job (include/recblr_hip.h)."""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p),
                ("exp_avg", ctypes.c_void_p), ("exp_avg_sq", ctypes.c_void_p),
                ("n", ctypes.c_int64)]


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam(params, lr, betas, eps, weight_decay) on rb_adam_step.
    Parameters and gradients must be contiguous fp32 CUDA tensors; a
    parameter without a gradient is skipped (as torch does)."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        if not 0.0 <= lr:
            raise ValueError(f"invalid learning rate {lr}")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid betas {betas}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                      weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            by_step = {}
            for p in group["params"]:
                if p.grad is None or p.numel() == 0:
                    continue   # torch.optim.Adam leaves an empty parameter as it is
                if (p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous()
                        or p.grad.dtype != torch.float32 or not p.grad.is_contiguous()):
                    raise ValueError("rb Adam: parameters and gradients must be contiguous fp32 "
                                     "CUDA tensors")
                if p.grad.is_sparse:
                    raise ValueError("rb Adam: sparse gradients are not supported")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                # a state loaded from torch.optim.Adam holds `step` as a tensor
                # (which hashes by identity): group launches by its value
                st["step"] = int(st["step"]) + 1
                by_step.setdefault(st["step"], []).append(p)
            for t, ps in by_step.items():
                bc1, bc2 = 1.0 - b1 ** t, 1.0 - b2 ** t
                for k in range(0, len(ps), MAX_ADAM_JOBS):
                    chunk = ps[k:k + MAX_ADAM_JOBS]
                    arr = (_AdamJob * len(chunk))()
                    for d, p in zip(arr, chunk):
                        st = self.state[p]
                        d.param, d.grad = p.data_ptr(), p.grad.data_ptr()
                        d.exp_avg, d.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
                        d.n = p.numel()
                    _lib.call("rb_adam_step", ctypes.addressof(arr), len(chunk),
                              float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                              float(group["weight_decay"]), float(bc1), float(bc2),
                              kernels._stream(chunk[0]))
        return loss


def native_ok(params) -> bool:
    """Whether every parameter meets rb_adam_step's requirements (contiguous
    fp32 CUDA tensors)."""
    return all(p.dtype == torch.float32 and p.is_cuda and p.is_contiguous() for p in params)


def make_adam(params, lr: float = 1e-3, weight_decay: float = 0.0, kind: str | None = None):
    """The training loop's Adam (RecBole's learner 'adam'): the native
    one-launch Adam, or torch.optim.Adam with RECBLR_ADAM=torch (kind
    overrides the variable).  Parameters the native kernel cannot take
    (CPU, non-fp32 or non-contiguous) fall back to torch.optim.Adam — the
    same semantics, checked against each other in tests/test_gpu_optim.py."""
    import os

    params = list(params)
    kind = kind or os.environ.get("RECBLR_ADAM", "native")
    if kind not in ("native", "torch"):
        raise ValueError(f"RECBLR_ADAM must be native or torch, got {kind!r}")
    if kind == "native" and native_ok(params):
        return Adam(params, lr=lr, weight_decay=weight_decay)
    fused = all(p.is_cuda and p.dtype == torch.float32 for p in params)
    return torch.optim.Adam(params, lr=lr, weight_decay=weight_decay, fused=fused or None)
