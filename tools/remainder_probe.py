import torch
dev = torch.device("cuda:0")
shapes = {"in.fwd": (128, 512), "in.dX": (512, 128), "gates.fwd": (256, 512), "gates.dX": (512, 256),
          "out.fwd": (256, 128), "out.dX": (128, 256), "w2.fwd": (512, 128), "w2.dX": (128, 512)}
rem = 8024
for name, (R, C) in shapes.items():
    a = torch.randn(rem, R, device=dev); w = torch.randn(C, R, device=dev); o = torch.empty(rem, C, device=dev)
    for _ in range(5): torch.mm(a, w.t(), out=o)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50): torch.mm(a, w.t(), out=o)
    e1.record(); e1.synchronize()
    t_mm = e0.elapsed_time(e1) / 50 * 1e3
    n = rem // 32 * 32
    e0.record()
    for _ in range(50):
        torch.linalg.vector_norm(a[:n].reshape(-1, 32 * R), ord=float("inf"), dim=1)
    e1.record(); e1.synchronize()
    t_rm = e0.elapsed_time(e1) / 50 * 1e3
    print(f"{name:10s} R={R:4d} C={C:4d} mm {t_mm:6.1f} us  rmax {t_rm:5.1f} us")
