"""Times the FeedForward activation GEMMs (rb_gemm_nt_h_act / _dact) against
the two-launch path at the bench's packed row count, and checks them bit for
bit against it; RECBLR_LIB selects a variant build (tools/ab_build.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from datamining_recblr_amd import kernels  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1000 for a, b in ev)
    return ts[reps // 2]


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(5)
    M, R, C, p, seed = 204632, 128, 512, 0.2, 99
    x = torch.randn(M, R, generator=g).to(dev)
    w1 = (torch.randn(C, R, generator=g) / R ** 0.5).to(dev)
    b1 = (0.1 * torch.randn(C, generator=g)).to(dev)
    da2 = torch.randn(M, R, generator=g).to(dev)
    w2 = (torch.randn(R, C, generator=g) / R ** 0.5).to(dev)
    wi1 = kernels.gemm_h_weight(w1)
    wi2 = kernels.gemm_h_weight(w2, transpose=True)
    rm = torch.empty((M + 31) // 32, device=dev)
    pre, act = kernels.gemm_nt_h_act(x, wi1, C, b1, seed, p, rmax=rm)
    da, db = kernels.gemm_nt_h_dact(da2, wi2, C, pre, seed, p, rmax=rm)
    du = kernels.gemm_nt_h(da2, wi2, C, rmax=rm)
    da_r, db_r = kernels.silu_dropout_bwd(pre, du, seed=seed, p=p, want_dbias=True)
    assert torch.equal(da, da_r), "dact differs"
    assert torch.equal(act, kernels.silu_dropout_fwd(pre, seed=seed, p=p)), "act differs"
    res = {
        "fwd_fused_us": timeit(lambda: kernels.gemm_nt_h_act(x, wi1, C, b1, seed, p, rmax=rm)),
        "fwd_gemm_us": timeit(lambda: kernels.gemm_nt_h(x, wi1, C, rmax=rm)),
        "fwd_act_us": timeit(lambda: kernels.silu_dropout_fwd(pre, seed=seed, p=p, bias=b1)),
        "bwd_fused_us": timeit(lambda: kernels.gemm_nt_h_dact(da2, wi2, C, pre, seed, p, rmax=rm)),
        "bwd_gemm_us": timeit(lambda: kernels.gemm_nt_h(da2, wi2, C, rmax=rm)),
        "bwd_act_us": timeit(lambda: kernels.silu_dropout_bwd(pre, du, seed=seed, p=p,
                                                              want_dbias=True)),
    }
    print(os.environ.get("RECBLR_LIB", "default"),
          {k: round(v, 1) for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
