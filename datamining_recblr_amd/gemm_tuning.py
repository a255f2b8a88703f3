"""Pinned hipBLASLt / rocBLAS solution choice for the encoder's projection GEMMs.

The BLAS heuristics pick a kernel per GEMM shape without timing it.  For the
tall-skinny fp32 projections of this encoder ([B*L, K] x [K, N], K, N in
{128, 256, 512}) several heuristic picks are 10-30% slower than the best
solution the libraries ship.  ``tuning/gemm_gfx950.csv`` is a PyTorch
TunableOp results table produced once on an MI355X (tuning run of bench.py,
``PYTORCH_TUNABLEOP_TUNING=1``); loading it with tuning *disabled* makes every
listed shape dispatch straight to its measured-best solution (no timing at run
time, deterministic) and leaves every other shape on the default heuristic.

The table carries validators (torch, HIP, hipBLASLt, rocBLAS versions and the
gfx arch); on a mismatch TunableOp refuses it and the defaults are used.
Set RECBLR_TUNED_GEMMS=0 to opt out.
"""
from __future__ import annotations

import os
import threading

import torch

__all__ = ["TABLE_PATH", "use_tuned_gemms", "tuned_gemms_active"]

TABLE_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "gemm_gfx950.csv")

_lock = threading.Lock()
_state = None  # None: not attempted; True/False: table loaded or not


def use_tuned_gemms(path: str = TABLE_PATH) -> bool:
    """Enable TunableOp in replay-only mode with the shipped table (idempotent).

    Returns True when the table was accepted.  Does nothing (returns False)
    without a GPU or with RECBLR_TUNED_GEMMS=0.  A user who already enabled
    TunableOp tuning keeps their own configuration."""
    global _state
    with _lock:
        if _state is not None:
            return _state
        _state = False
        if os.environ.get("RECBLR_TUNED_GEMMS", "1") == "0" or not torch.cuda.is_available():
            return False
        tun = torch.cuda.tunable
        if tun.is_enabled() and tun.tuning_is_enabled():
            return False
        if not os.path.exists(path):
            return False
        tun.tuning_enable(False)
        tun.record_untuned_enable(False)
        tun.enable(True)
        _state = bool(tun.read_file(path))
        if not _state:
            tun.enable(False)
        return _state


def tuned_gemms_active() -> bool:
    return bool(_state)
