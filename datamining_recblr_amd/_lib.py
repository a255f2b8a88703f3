"""ctypes binding of the C-ABI in include/recblr_hip.h.

The shared library is built in-tree by ``datamining_recblr_amd.build`` (or
``__graft_entry__.build()``) as ``datamining_recblr_amd/lib/libdmrecblr.so``.
There is no fallback: if the library is missing, every product entry point
raises ``RecBLRNativeError``.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# RECBLR_LIB points at an alternative build of the same sources (A/B timing
# of compile-time variants, e.g. tools/ab_build.sh); the default is the in-tree build
LIB_PATH = os.environ.get("RECBLR_LIB") or os.path.join(_HERE, "lib", "libdmrecblr.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "recblr_hip.h")

RB_EINVAL = -1
RB_TILE = 16
ABI_VERSION = 44

_i64 = ctypes.c_int64
_fp = ctypes.c_void_p  # device pointers are passed as integers
_f32 = ctypes.c_float
_u64 = ctypes.c_uint64

# name -> (restype, argtypes); kept in the order of include/recblr_hip.h
SIGNATURES = {
    "rb_version": (ctypes.c_int, []),
    "rb_last_error_string": (ctypes.c_char_p, []),
    "rb_num_kernels": (ctypes.c_int, []),
    "rb_scan_fwd": (ctypes.c_int, [_fp, _fp, _fp, _i64, _i64, _i64, _fp]),
    "rb_scan_bwd": (ctypes.c_int, [_fp, _fp, _fp, _fp, _fp, _i64, _i64, _i64, _fp]),
    "rb_conv_silu_fwd": (ctypes.c_int, [_fp, _i64, _fp, _fp, _fp, _i64, _i64, _i64, _i64, _i64, _fp, _fp]),
    "rb_conv_silu_fwd_rows": (ctypes.c_int, [_fp, _i64, _fp, _fp, _fp, _i64, _i64, _i64, _i64,
                                             _fp, _fp]),
    "rb_conv_silu_fwd_rows_bf16": (ctypes.c_int, [_fp, _i64, _fp, _fp, _fp, _i64, _i64, _i64,
                                                  _i64, _fp, _fp]),
    "rb_conv_silu_bwd": (ctypes.c_int, [_fp, _i64, _fp, _fp, _fp, _fp, _fp, _i64, _fp, _fp,
                                        _i64, _i64, _i64, _i64, _fp, _fp]),
    "rb_gate_scan_fwd": (ctypes.c_int, [_fp, _i64, _fp, _i64, _fp, _i64, _fp, _fp, _fp, _i64, _fp,
                                        _i64, _fp, _i64, _i64, _i64, _fp, _fp]),
    "rb_gate_scan_fwd_last": (ctypes.c_int, [_fp, _i64, _fp, _i64, _fp, _i64, _fp, _fp, _fp,
                                             _i64, _fp, _fp, _i64, _i64, _i64, _fp, _fp, _fp]),
    "rb_gate_scan_bwd_last": (ctypes.c_int, [_fp, _i64, _fp, _i64, _fp, _i64, _fp, _fp, _fp,
                                             _fp, _fp, _i64, _fp, _i64, _fp, _i64, _fp, _fp,
                                             _i64, _i64, _i64, _fp, _fp, _fp]),
    "rb_gate_scan_bwd": (ctypes.c_int, [_fp, _i64, _fp, _i64, _fp, _i64, _fp, _fp, _fp, _fp, _fp,
                                        _i64, _fp, _i64, _fp, _i64, _fp, _fp, _i64, _i64, _i64,
                                        _fp, _fp]),
    "rb_pad_prefix_fwd": (ctypes.c_int, [_fp, _fp, _fp, _fp, _fp, _i64, _i64, _i64, _fp, _fp, _fp]),
    "rb_pad_prefix_bwd": (ctypes.c_int, [_fp, _fp, _fp, _fp, _fp, _i64, _i64, _i64, _fp, _fp, _fp,
                                         _fp, _fp, _fp, ctypes.c_int, _fp]),
    "rb_add_ln_fwd": (ctypes.c_int, [_fp, _fp, _i64, _fp, _u64, _f32, _fp, _fp, _fp, _f32, _fp,
                                     _fp, _fp, _fp, _i64, _i64, _fp]),
    "rb_row_num_parts": (ctypes.c_int64, [_i64, _i64]),
    "rb_add_ln_bwd": (ctypes.c_int, [_fp, _fp, _fp, _fp, _fp, _fp, _u64, _f32, _fp, _fp, _fp, _fp,
                                     _fp, _i64, _i64, _i64, _fp]),
    "rb_add_ln_bwd2": (ctypes.c_int, [_fp, _fp, _fp, _fp, _fp, _fp, _fp, _u64, _f32, _fp, _fp, _fp, _fp,
                                     _fp, _i64, _i64, _i64, _fp]),
    "rb_silu_dropout_fwd": (ctypes.c_int, [_fp, _fp, _fp, _u64, _f32, _fp, _i64, _i64, _fp]),
    "rb_silu_dropout_bwd": (ctypes.c_int, [_fp, _fp, _fp, _u64, _f32, _fp, _fp, _fp, _i64, _i64,
                                           _i64, _fp]),
    "rb_dropout_mask": (ctypes.c_int, [_u64, _f32, _fp, _i64, _fp]),
    "rb_embedding_bwd_workspace": (ctypes.c_int64, [_i64, _i64, _i64]),
    "rb_embedding_bwd": (ctypes.c_int, [_fp, _fp, _i64, _i64, _i64, _i64, _fp, _fp, _i64, _fp]),
    "rb_embedding_bwd_plan": (ctypes.c_int, [_fp, _i64, _i64, _i64, _fp, _i64, _fp]),
    "rb_embedding_bwd_apply": (ctypes.c_int, [_fp, _i64, _i64, _i64, _i64, _fp, _fp, _i64, _fp]),
    "rb_colsum": (ctypes.c_int, [_fp, _i64, _i64, _i64, _i64, _i64, _fp, _fp]),
    "rb_colsum_chunked": (ctypes.c_int, [_fp, _i64, _i64, _i64, _i64, _i64, _fp, _fp, _i64, _fp,
                                         _fp]),
    "rb_item_ce_workspace": (ctypes.c_int64, [_i64, _i64, _i64]),
    "rb_item_ce_fwd": (ctypes.c_int, [_fp, _fp, _fp, _i64, _i64, _i64, _fp, _fp, _fp, _i64, _fp]),
    "rb_item_ce_bwd": (ctypes.c_int, [_fp, _fp, _fp, _fp, _fp, _i64, _i64, _i64, _fp, _fp, _fp,
                                      _i64, _fp]),
    "rb_item_split_h": (ctypes.c_int, [_fp, _i64, _i64, _fp, _fp, _fp, _fp]),
    "rb_item_ce_fwd_h": (ctypes.c_int, [_fp, _fp, _fp, _fp, _fp, _i64, _i64, _i64, _fp, _fp, _fp,
                                        _i64, _fp]),
    "rb_item_ce_probs_h": (ctypes.c_int, [_fp, _fp, _fp, _fp, _fp, _fp, _fp, _i64, _i64, _i64,
                                          _i64, _fp, _i64, _fp]),
    "rb_item_ce_probs_h_t": (ctypes.c_int, [_fp, _fp, _fp, _fp, _fp, _fp, _fp, _i64, _i64, _i64,
                                            _i64, _fp, _i64, _fp, _fp]),
    "rb_item_ce_probs_h_both": (ctypes.c_int, [_fp, _fp, _fp, _fp, _fp, _fp, _fp, _i64, _i64,
                                               _i64, _i64, _fp, _i64, _fp, _i64, _fp, _fp, _fp]),
    "rb_group_absmax": (ctypes.c_int, [_fp, _i64, _i64, _i64, _fp, _fp]),
    "rb_item_rank_workspace": (ctypes.c_int64, [_i64, _i64, _i64]),
    "rb_item_rank": (ctypes.c_int, [_fp, _fp, _fp, _i64, _i64, _i64, _i64, _fp, _fp, _fp, _i64,
                                    _fp]),
    "rb_item_ce_probs": (ctypes.c_int, [_fp, _fp, _fp, _fp, _fp, _i64, _i64, _i64, _i64, _fp, _i64,
                                        _fp]),
    "rb_item_scores": (ctypes.c_int, [_fp, _fp, _i64, _i64, _i64, _fp, _fp]),
    "rb_scan_fwd_bf16": (ctypes.c_int, [_fp, _fp, _fp, _i64, _i64, _i64, _fp]),
    "rb_scan_bwd_bf16": (ctypes.c_int, [_fp, _fp, _fp, _fp, _fp, _i64, _i64, _i64, _fp]),
    "rb_conv_silu_fwd_bf16": (ctypes.c_int, [_fp, _i64, _fp, _fp, _fp, _i64, _i64, _i64, _i64,
                                             _i64, _fp, _fp]),
    "rb_conv_silu_bwd_bf16": (ctypes.c_int, [_fp, _i64, _fp, _fp, _fp, _fp, _fp, _i64, _fp, _fp,
                                             _i64, _i64, _i64, _i64, _fp, _fp]),
    "rb_gate_scan_fwd_bf16": (ctypes.c_int, [_fp, _i64, _fp, _i64, _fp, _i64, _fp, _fp, _fp,
                                             _i64, _fp, _i64, _fp, _i64, _i64, _i64, _fp, _fp]),
    "rb_gate_scan_bwd_bf16": (ctypes.c_int, [_fp, _i64, _fp, _i64, _fp, _i64, _fp, _fp, _fp, _fp,
                                             _fp, _i64, _fp, _i64, _fp, _i64, _fp, _fp, _i64,
                                             _i64, _i64, _fp, _fp]),
    "rb_pack_plan": (ctypes.c_int, [_fp, _i64, _fp, _fp, _i64, _i64, _fp, _fp, _fp, _fp, _fp]),
    "rb_gemm_h_weight_bytes": (ctypes.c_int64, [_i64, _i64]),
    "rb_gemm_nt_h_mode": (ctypes.c_int, [ctypes.c_int]),
    "rb_gemm_nt_h_ln": (ctypes.c_int, [_fp, _i64, _i64, _i64, _fp, _i64, _fp, _fp, _fp, _fp, _f32,
                                       _u64, _f32, _fp, _fp, _fp, _fp, _i64, _fp, _fp]),
    "rb_gemm_h_split_weights": (ctypes.c_int, [_fp, _i64, _fp]),
    "rb_gemm_nt_h": (ctypes.c_int, [_fp, _i64, _i64, _i64, _fp, _i64, _fp, _fp, _i64, ctypes.c_int,
                                    _fp, _fp]),
    "rb_gemm_nt_h_act": (ctypes.c_int, [_fp, _i64, _i64, _i64, _fp, _i64, _fp, _fp, _i64, _fp,
                                        _fp, _u64, _f32, _fp]),
    "rb_adam_step": (ctypes.c_int, [_fp, _i64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double, _fp]),
    "rb_gemm_nt_h_dact_parts": (_i64, []),
    "rb_gemm_nt_h_dact": (ctypes.c_int, [_fp, _i64, _i64, _i64, _fp, _i64, _fp, _i64, _fp, _fp,
                                         _u64, _f32, _fp, _i64, _fp]),
    "rb_gemm_bf16_weight_image": (ctypes.c_int, [_fp, _i64, _i64, _i64, ctypes.c_int, _fp, _fp]),
    "rb_gemm_nt_bf16": (ctypes.c_int, [_fp, _i64, _i64, _i64, _fp, _i64, _fp, _fp, _i64, _fp]),
    "rb_gemm_tn_h": (ctypes.c_int, [_fp, _i64, _fp, _i64, _i64, _i64, _i64, _fp, _fp, _fp, _i64,
                                    _fp]),
    "rb_gemm_tn_hs": (ctypes.c_int, [_fp, _i64, _fp, _i64, _i64, _i64, _i64, _fp, ctypes.c_int, _fp]),
}


class RecBLRNativeError(RuntimeError):
    """The HIP extension is missing, failed to load, or a kernel call failed."""


# the experimental library (experimental/recblr_exp.h: opt-in kernels that
# measured slower than the default path; never loaded unless requested)
EXP_SIGNATURES = {
    "rb_exp_version": (ctypes.c_int, []),
    "rb_exp_last_error_string": (ctypes.c_char_p, []),
    "rb_grl_fwd": (ctypes.c_int, [_fp, _i64, _fp, _i64, _fp, _fp, _fp, _fp, _fp, _fp, _i64, _i64,
                                  _i64, _i64, _fp, _i64, _fp, _fp, _fp, _fp, _i64, _fp, _fp,
                                  _i64, _fp]),
    "rb_grl_bwd": (ctypes.c_int, [_fp, _i64, _fp, _i64, _fp, _fp, _fp, _fp, _fp, _fp, _fp, _i64,
                                  _i64, _i64, _i64, _fp, _i64, _fp, _fp, _fp, _i64, _fp, _fp,
                                  _fp, _fp, _fp, _fp, _fp]),
}

# the probe library (probes/recblr_probe.h: bench.py's measurement aids)
PROBE_SIGNATURES = {
    "rb_probe_gemm_pattern": (ctypes.c_int, [_fp, _i64, _i64, _fp, _i64, _fp]),
    "rb_probe_gate_bwd_pattern": (ctypes.c_int, [_fp, _i64, _fp, _i64, _fp, _i64, _fp, _fp, _i64,
                                                 _fp, _i64, _fp, _i64, _i64, _i64, _i64, _fp,
                                                 _fp]),
}

_lock = threading.Lock()
_lib = None
_probe = None
_exp = None


def load(path: str | None = None) -> ctypes.CDLL:
    """Load (once) and return the native library with typed prototypes."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RecBLRNativeError(
                f"HIP extension not built: {p} is missing. Run "
                "`python -m datamining_recblr_amd.build` (hipcc --offload-arch=gfx950)."
            )
        try:
            lib = ctypes.CDLL(p)
        except OSError as exc:  # pragma: no cover - depends on the host
            raise RecBLRNativeError(f"failed to load {p}: {exc}") from exc
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.rb_version() != ABI_VERSION:
            raise RecBLRNativeError(
                f"ABI mismatch: library {lib.rb_version()} vs binding {ABI_VERSION}; rebuild")
        if path is None:
            _lib = lib
        return lib


_fns = {}
_failure_hooks = []


def on_failure(hook) -> None:
    """Register hook() to run whenever a C-ABI call returns an error (device
    state cached by the Python side, e.g. the column sums' ticket counters,
    is dropped rather than trusted after a failure)."""
    _failure_hooks.append(hook)


def call(name: str, *args) -> None:
    """Invoke a C-ABI entry point and raise on a non-zero status."""
    fn = _fns.get(name)
    if fn is None:
        fn = _fns[name] = getattr(load(), name)
    rc = fn(*args)
    if rc != 0:
        for hook in _failure_hooks:
            hook()
        lib = load()
        msg = lib.rb_last_error_string()
        msg = msg.decode() if msg else ""
        kind = "invalid argument" if rc == RB_EINVAL else f"hipError {rc}"
        raise RecBLRNativeError(f"{name} failed ({kind}): {msg}")


def load_probe() -> ctypes.CDLL:
    """The probe library (lib/libdmrecblr_probe.so): measurement aids for
    bench.py, never on the model's path."""
    global _probe
    with _lock:
        if _probe is not None:
            return _probe
        p = os.path.join(os.path.dirname(LIB_PATH), "libdmrecblr_probe.so")
        if not os.path.exists(p):
            raise RecBLRNativeError(f"probe library not built: {p} is missing. Run "
                                    "`python -m datamining_recblr_amd.build`.")
        lib = ctypes.CDLL(p)
        for name, (res, args) in PROBE_SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        lib.rb_probe_last_error_string.restype = ctypes.c_char_p
        _probe = lib
        return lib


def call_probe(name: str, *args) -> None:
    """Invoke a probe-library entry point and raise on a non-zero status."""
    lib = load_probe()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.rb_probe_last_error_string()
        raise RecBLRNativeError(f"{name} failed ({rc}): {msg.decode() if msg else ''}")


def load_exp() -> ctypes.CDLL:
    """The experimental library (lib/libdmrecblr_exp.so, experimental/
    recblr_exp.h): the opt-in fused GatedRecurrentLayer kernels.  Loaded only
    when one of them is requested; the default path never loads it."""
    global _exp
    with _lock:
        if _exp is not None:
            return _exp
        p = os.path.join(os.path.dirname(LIB_PATH), "libdmrecblr_exp.so")
        if not os.path.exists(p):
            raise RecBLRNativeError(f"experimental library not built: {p} is missing. Run "
                                    "`python -m datamining_recblr_amd.build`.")
        lib = ctypes.CDLL(p)
        for name, (res, args) in EXP_SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.rb_exp_version() != ABI_VERSION:
            raise RecBLRNativeError(f"experimental library ABI {lib.rb_exp_version()} vs "
                                    f"{ABI_VERSION}; rebuild")
        _exp = lib
        return lib


def call_exp(name: str, *args) -> None:
    """Invoke an experimental-library entry point and raise on a non-zero status."""
    lib = load_exp()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        for hook in _failure_hooks:
            hook()
        msg = lib.rb_exp_last_error_string()
        kind = "invalid argument" if rc == RB_EINVAL else f"hipError {rc}"
        raise RecBLRNativeError(f"{name} failed ({kind}): {msg.decode() if msg else ''}")
