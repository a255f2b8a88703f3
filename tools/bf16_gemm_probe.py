"""configs[4]'s six NT projection GEMMs (M = 2,097,152 rows) one shape at a
time: our bf16 kernel (rb_gemm_nt_bf16) against torch's bf16 GEMMs
(hipBLASLt), median of 7 HIP-event timings, with each shape's algorithmic
TFLOP/s and GB/s (the weight gradients run on hipBLASLt in every mode)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from datamining_recblr_amd import kernels  # noqa: E402


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


if __name__ == "__main__":
    t0 = time.time()
    main(*(int(v) for v in sys.argv[1:]))
    print(f"done in {time.time() - t0:.1f} s")
