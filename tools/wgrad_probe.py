import sys, torch
sys.path.insert(0, '.')
from datamining_recblr_amd import linear, gemm_tuning
print("tuned:", gemm_tuning.use_tuned_gemms())
dev = torch.device('cuda')
M = 204169
def bench(fn, reps=10):
    fn(); torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    ts.sort(); return ts[len(ts)//2] * 1e3
for N, K in [(512, 256), (512, 128), (128, 512), (128, 256), (256, 512), (256, 128)]:
    dy = torch.randn(M, N, device=dev); x = torch.randn(M, K, device=dev)
    f = 2.0 * M * N * K
    row = []
    for sp in (16, 32, 48, 64, 96, 128, 256):
        t = bench(lambda: linear.wgrad(dy, x, splits=sp))
        row.append(f"{sp}:{t:6.1f}us/{f/t/1e6:5.1f}TF")
    print(f"dW [{N}x{K}]", " ".join(row), flush=True)
