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
