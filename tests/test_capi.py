"""The C-ABI library loads on a CPU-only host and exports exactly what
include/recblr_hip.h declares (no compute call is made here)."""
import ctypes
import re

from datamining_recblr_amd import _lib


def header_functions():
    text = open(_lib.HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return re.findall(r"\b(rb_[a-z0-9_]+)\s*\(", text)


def test_header_declares_expected_entry_points():
    names = header_functions()
    assert len(names) == len(set(names))
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)
    for must in ("rb_scan_fwd", "rb_scan_bwd", "rb_conv_silu_fwd", "rb_conv_silu_bwd",
                 "rb_gate_scan_fwd", "rb_gate_scan_bwd", "rb_version", "rb_last_error_string"):
        assert must in names


def test_library_loads_and_exports_every_symbol():
    lib = _lib.load()
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for name in header_functions():
        assert hasattr(raw, name), name
    assert lib.rb_version() == _lib.ABI_VERSION
    assert lib.rb_num_kernels() > 0


def test_tile_constant_matches_header():
    text = open(_lib.HEADER_PATH).read()
    assert re.search(r"#define RB_TILE (\d+)", text).group(1) == str(_lib.RB_TILE)
    assert re.search(r"#define RB_EINVAL \((-?\d+)\)", text).group(1) == str(_lib.RB_EINVAL)


def test_argument_errors_are_reported_without_touching_the_gpu():
    lib = _lib.load()
    # null pointers are rejected before any HIP call
    rc = lib.rb_scan_fwd(None, None, None, 1, 1, 1, None)
    assert rc == _lib.RB_EINVAL
    assert b"null" in lib.rb_last_error_string()
    rc = lib.rb_conv_silu_fwd(1, 4, 1, 1, 1, 4, 1, 1, 4, 9, None, None)
    assert rc == _lib.RB_EINVAL
    assert b"K must be" in lib.rb_last_error_string()
    rc = lib.rb_gate_scan_fwd(1, 3, 1, 4, 1, 4, 1, 0, 0, 0, 1, 4, 1, 1, 1, 4, None, None)
    assert rc == _lib.RB_EINVAL   # rg row stride < 2H


def test_row_conv_and_batched_split_argument_errors():
    """ABI 18/19 entry points validate before any HIP call."""
    lib = _lib.load()
    rc = lib.rb_conv_silu_fwd_rows(1, 4, 1, 1, 1, 4, 8, 4, 4, None, None)
    assert rc == _lib.RB_EINVAL and b"null" in lib.rb_last_error_string()
    rc = lib.rb_conv_silu_fwd_rows(1, 4, 1, 1, 1, 4, 8, 4, 9, 1, None)
    assert rc == _lib.RB_EINVAL and b"K must be" in lib.rb_last_error_string()
    from datamining_recblr_amd import kernels

    jobs = (kernels._SplitJob * 1)()
    jobs[0].W, jobs[0].ldw, jobs[0].C, jobs[0].R, jobs[0].transpose, jobs[0].Wf = 16, 40, 32, 40, 0, 16
    rc = lib.rb_gemm_h_split_weights(ctypes.addressof(jobs), 1, None)
    assert rc == _lib.RB_EINVAL and b"multiple of" in lib.rb_last_error_string()   # R % 16
    rc = lib.rb_gemm_h_split_weights(ctypes.addressof(jobs), 0, None)
    assert rc == _lib.RB_EINVAL
    rc = lib.rb_gemm_h_split_weights(ctypes.addressof(jobs), 33, None)
    assert rc == _lib.RB_EINVAL


def test_f16_item_ce_argument_errors():
    """ABI 24 entry points (the CE on split images) validate before any HIP call."""
    lib = _lib.load()
    rc = lib.rb_item_split_h(None, 4, 128, 16, 16, None, None)
    assert rc == _lib.RB_EINVAL and b"null" in lib.rb_last_error_string()
    rc = lib.rb_item_split_h(16, 4, 48, 16, 16, None, None)
    assert rc == _lib.RB_EINVAL and b"d must be" in lib.rb_last_error_string()
    rc = lib.rb_item_split_h(8, 4, 128, 16, 16, None, None)     # 8 is not 16-B aligned
    assert rc == _lib.RB_EINVAL and b"aligned" in lib.rb_last_error_string()
    rc = lib.rb_item_ce_fwd_h(16, None, 16, 16, 16, 4, 8, 128, 16, 16, 16, 1 << 20, None)
    assert rc == _lib.RB_EINVAL and b"exponent" in lib.rb_last_error_string()
    rc = lib.rb_item_ce_fwd_h(16, 16, 16, 16, 16, 4, 8, 100, 16, 16, 16, 1 << 20, None)
    assert rc == _lib.RB_EINVAL and b"d must be" in lib.rb_last_error_string()
    rc = lib.rb_item_ce_probs_h(16, 16, 16, 16, 16, 16, 16, 4, 8, 128, 0, 16, 7, None)
    assert rc == _lib.RB_EINVAL and b"ld < V" in lib.rb_last_error_string()


def test_probe_library_is_separate_and_exports_its_header():
    """bench.py's measurement aids live in their own library
    (probes/recblr_probe.h, lib/libdmrecblr_probe.so): the product library
    exports none of them, the probe library exports exactly its header's."""
    import os
    hdr = os.path.join(os.path.dirname(_lib.__file__), "probes", "recblr_probe.h")
    text = re.sub(r"/\*.*?\*/", "", open(hdr).read(), flags=re.S)
    names = re.findall(r"\b(rb_[a-z0-9_]+)\s*\(", text)
    assert set(names) == set(_lib.PROBE_SIGNATURES) | {"rb_probe_last_error_string"}
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert not hasattr(raw, n), n
    probe = _lib.load_probe()
    for n in names:
        assert hasattr(probe, n), n
    # argument errors are reported without touching the GPU
    try:
        _lib.call_probe("rb_probe_gemm_pattern", None, 1, 4, None, 4, None)
    except _lib.RecBLRNativeError as e:
        assert "null pointer" in str(e)
    else:
        raise AssertionError("null pointers accepted")


def test_tn_weight_gradient_rejects_row_chunks_of_2_gib():
    """rb_gemm_tn_h addresses a row chunk with 32-bit offsets through a buffer
    descriptor: a chunk spanning 2 GiB of an operand is an argument error
    naming the limit (checked before any HIP call), never a silent wrap."""
    lib = _lib.load()
    M, N, K = 1 << 22, 128, 128
    # 8 splits of 2^22 rows: 2^19-row chunks; at a 2^13-float row stride of dY
    # a chunk spans 2^19 x 32 KiB = 16 GiB
    rc = lib.rb_gemm_tn_h(16, 1 << 13, 16, K, M, N, K, 16, 16, 16, 8, None)
    assert rc == _lib.RB_EINVAL and b"2 GiB" in lib.rb_last_error_string()


def test_experimental_library_is_separate_and_exports_its_header():
    """The opt-in fused GatedRecurrentLayer kernels (RECBLR_FUSED_GRL*) live
    in their own library (experimental/recblr_exp.h, lib/libdmrecblr_exp.so):
    the product library exports none of them, the experimental library
    exactly its header's, at the product's ABI version; argument errors are
    reported without touching the GPU."""
    import os
    hdr = os.path.join(os.path.dirname(_lib.__file__), "experimental", "recblr_exp.h")
    text = re.sub(r"/\*.*?\*/", "", open(hdr).read(), flags=re.S)
    names = re.findall(r"\b(rb_[a-z0-9_]+)\s*\(", text)
    assert set(names) == set(_lib.EXP_SIGNATURES)
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert not hasattr(raw, n), n
    exp = _lib.load_exp()
    assert exp.rb_exp_version() == _lib.ABI_VERSION
    try:
        _lib.call_exp("rb_grl_fwd", *[0 if t is ctypes.c_int64 else None
                                      for t in _lib.EXP_SIGNATURES["rb_grl_fwd"][1]])
    except _lib.RecBLRNativeError as e:
        assert "null pointer" in str(e)
    else:
        raise AssertionError("null pointers accepted")
