"""Experiment: the 1x1 compress conv (models.py:165) as MIOpen conv vs batched GEMM, fp32.
Not product code."""
import time

import torch

dev = torch.device("cuda:0")


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


for name, Nt, C, HW in [("cfg2", 128, 512, 32), ("ns", 256, 512, 32), ("cfg3", 256, 1280, 8), ("cfg4", 64, 2048, 8),
                        ("cfg5", 512, 1024, 16)]:
    torch.manual_seed(0)
    x = torch.randn(Nt, 2 * C, HW, HW, device=dev)
    conv = torch.nn.Conv2d(2 * C, C, 1).to(dev)
    W = conv.weight.view(C, 2 * C)
    flop = 2.0 * Nt * HW * HW * 2 * C * C
    with torch.no_grad():
        t_conv = timeit(lambda: conv(x))
        t_mm = timeit(lambda: torch.baddbmm(conv.bias.view(1, C, 1), W.expand(Nt, C, 2 * C), x.view(Nt, 2 * C, -1)))
        t_mm2 = timeit(lambda: torch.matmul(W, x.view(Nt, 2 * C, -1)))
        ref = conv(x)
        alt = torch.baddbmm(conv.bias.view(1, C, 1), W.expand(Nt, C, 2 * C), x.view(Nt, 2 * C, -1)).view_as(ref)
        err = float((ref - alt).abs().max() / ref.abs().max())
    print(f"{name}: Nt={Nt} C={C} {HW}x{HW}  conv {t_conv*1e6:8.1f} us ({flop/t_conv/1e12:6.1f} TF)  "
          f"baddbmm {t_mm*1e6:8.1f} us ({flop/t_mm/1e12:6.1f} TF)  matmul {t_mm2*1e6:8.1f} us  relerr {err:.2e}",
          flush=True)
