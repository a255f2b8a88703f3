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
    """Records every launch of the split-bf16 GEMM (kernels.gemm_nt, the
    rb_gemm_nt C-ABI entry) as (M, R, C): tests use it to assert that the
    path they claim to check actually ran the kernel."""
    from datamining_recblr_amd import kernels

    calls = []
    orig = kernels.gemm_nt

    def counted(a, wf, C, *args, **kw):
        calls.append((a.shape[0], a.shape[1], C))
        return orig(a, wf, C, *args, **kw)

    monkeypatch.setattr(kernels, "gemm_nt", counted)
    return calls
