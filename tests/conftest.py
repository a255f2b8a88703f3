import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line(
        "markers", "experimental: the opt-in experimental library's kernels (not the product "
        "path); skipped unless RECBLR_TEST_EXPERIMENTAL=1")


def pytest_collection_modifyitems(config, items):
    """Experimental kernels (datamining_recblr_amd/experimental/, slower than the
    product path and off by default) stay out of the default GPU suite."""
    if os.environ.get("RECBLR_TEST_EXPERIMENTAL") == "1":
        return
    skip = pytest.mark.skip(reason="experimental kernels: set RECBLR_TEST_EXPERIMENTAL=1")
    for item in items:
        if item.get_closest_marker("experimental") is not None:
            item.add_marker(skip)


def load_golden(name):
    import torch

    return torch.load(os.path.join(GOLDEN, name), weights_only=True)["cases"]


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch.cuda.is_available() is False")
    return torch.device("cuda:0")


@pytest.fixture
def split_gemm_calls(monkeypatch):
    """Records every launch of the f16x3 split-operand GEMM (kernels.gemm_nt_h
    / rb_gemm_nt_h and its fused-epilogue variants kernels.gemm_nt_h_act /
    gemm_nt_h_dact / gemm_nt_h_ln) as (M, R, C): tests use it to assert that
    the path they claim to check actually ran the kernel."""
    from datamining_recblr_amd import kernels

    calls = []
    for name in ("gemm_nt_h", "gemm_nt_h_act", "gemm_nt_h_dact", "gemm_nt_h_ln"):
        orig = getattr(kernels, name)

        def counted(a, wf, C, *args, _orig=orig, **kw):
            calls.append((a.shape[0], a.shape[1], C))
            return _orig(a, wf, C, *args, **kw)

        monkeypatch.setattr(kernels, name, counted)
    return calls


@pytest.fixture
def tn_gemm_calls(monkeypatch):
    """Records every launch of the f16 weight-gradient kernel
    (kernels.gemm_tn_h / rb_gemm_tn_h) as (M, N, K) of dW[N, K] = dY[M, N]^T
    X[M, K]: tests use it to assert the weight gradients they check ran on it
    (it needs M >= linear.MIN_ROWS_FOR_SPLIT and the rmax side outputs)."""
    from datamining_recblr_amd import kernels

    calls = []
    orig = kernels.gemm_tn_h

    def counted(dy, x, ymax, xmax, *args, **kw):
        calls.append((dy.shape[0], dy.shape[1], x.shape[1]))
        return orig(dy, x, ymax, xmax, *args, **kw)

    monkeypatch.setattr(kernels, "gemm_tn_h", counted)
    return calls
