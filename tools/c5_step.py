"""One configs[4] GatedRecurrentLayer fwd+bwd step (B=1024, L=2048, d=256,
bf16 activations), repeated: for rocprof kernel summaries of the C5 step."""
import sys
import time

import torch

sys.path.insert(0, ".")
from datamining_recblr_amd.model import GatedRecurrentLayer  # noqa: E402


def main(steps=4, B=1024):
    dev = torch.device("cuda:0")
    L, d = 2048, 256
    torch.manual_seed(2020)
    layer = GatedRecurrentLayer(d_model=d).to(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, L, d, device=dev, generator=g).to(torch.bfloat16).requires_grad_()
    gy = torch.randn(B, L, d, device=dev, generator=g).to(torch.bfloat16)
    for i in range(steps + 1):
        if i == 1:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        layer.zero_grad(set_to_none=True)
        x.grad = None
        layer(x).backward(gy)
    torch.cuda.synchronize()
    print(f"C5 step {1e3 * (time.perf_counter() - t0) / steps:.2f} ms (B={B})")


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
