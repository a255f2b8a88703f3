import torch, sys
sys.path.insert(0, '/root/repo')
from datamining_recblr_amd.gemm_tuning import use_tuned_gemms
print('tuned', use_tuned_gemms())
dev='cuda'
def t(fn, reps=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1)/reps*1e3
M=409600
for K,N in [(128,512),(256,512),(512,128),(256,128)]:
    x=torch.randn(M,K,device=dev); w=torch.randn(N,K,device=dev); b=torch.randn(N,device=dev)
    fl=2*M*K*N
    a=t(lambda: torch.addmm(b,x,w.t())); c=t(lambda: torch.mm(x,w.t()))
    print(f"K={K} N={N}: addmm(bias) {a:7.1f}us {fl/a/1e6:6.1f}TF   mm {c:7.1f}us {fl/c/1e6:6.1f}TF")
