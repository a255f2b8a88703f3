"""configs[4]'s nine projection GEMMs (M = 2,097,152 rows) one shape at a
time: our bf16 kernels (rb_gemm_nt_bf16 / rb_gemm_tn_bf16 + column sum)
against torch's bf16 GEMMs (hipBLASLt), median of 7 HIP-event timings, with
each shape's algorithmic TFLOP/s and GB/s."""
import sys
import time

import torch

sys.path.insert(0, ".")
from datamining_recblr_amd import kernels, linear  # noqa: E402


def med(fn, reps=7):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main(M=2097152):
    dev = torch.device("cuda:0")
    d, H = 256, 512
    g = torch.Generator(device=dev).manual_seed(1)
    nt = {"in.fwd": (d, 2 * H), "gates.fwd": (H, 2 * H), "out.fwd": (H, d),
          "in.dX": (2 * H, d), "gates.dX": (2 * H, H), "out.dX": (d, H)}
    for name, (R, C) in nt.items():
        a = torch.randn(M, R, device=dev, generator=g).to(torch.bfloat16)
        w = torch.randn(C, R, device=dev, generator=g) * R ** -0.5
        img = kernels.bf16_weight_image(w)
        wb = w.to(torch.bfloat16)
        t_own = med(lambda: kernels.gemm_nt_bf16(a, img, C))
        t_ref = med(lambda: a @ wb.t())
        fl, by = 2 * M * R * C, 2 * M * (R + C)
        print(f"NT {name:10s} R={R:5d} C={C:5d}: own {t_own:7.3f} ms ({fl / t_own / 1e9:6.0f} TF/s, "
              f"{by / t_own / 1e6:6.0f} GB/s)  torch {t_ref:7.3f} ms", flush=True)
        if name.endswith(".fwd"):
            b = torch.randn(C, device=dev, generator=g)
            bb = b.to(torch.bfloat16)
            t_own = med(lambda: kernels.gemm_nt_bf16(a, img, C, bias=b))
            t_ref = med(lambda: torch.addmm(bb, a, wb.t()))
            print(f"NT {name + '+b':10s} R={R:5d} C={C:5d}: own {t_own:7.3f} ms "
                  f"({fl / t_own / 1e9:6.0f} TF/s, {by / t_own / 1e6:6.0f} GB/s)  torch {t_ref:7.3f} ms",
                  flush=True)
        del a
    tn = {"in.dW": (2 * H, d), "gates.dW": (2 * H, H), "out.dW": (d, H)}
    for name, (N, K) in tn.items():
        dy = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        t_own = med(lambda: linear.wgrad(dy, x))
        prev = linear.set_bf16_gemm(False)
        t_ref = med(lambda: linear.wgrad(dy, x))
        linear.set_bf16_gemm(prev)
        fl, by = 2 * M * N * K, 2 * M * (N + K)
        print(f"TN {name:10s} N={N:5d} K={K:5d}: own {t_own:7.3f} ms ({fl / t_own / 1e9:6.0f} TF/s, "
              f"{by / t_own / 1e6:6.0f} GB/s)  torch {t_ref:7.3f} ms", flush=True)
        del dy, x


if __name__ == "__main__":
    t0 = time.time()
    main(*(int(v) for v in sys.argv[1:]))
    print(f"done in {time.time() - t0:.1f} s")
