"""Experiment: 1x1 compress conv forward+backward, MIOpen conv vs batched-GEMM formulations, fp32.
Not product code."""
import time

import torch

dev = torch.device("cuda:0")


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


for name, Nt, C, HW in [("ns", 256, 512, 32), ("cfg3", 256, 1280, 8), ("cfg5", 512, 1024, 16)]:
    torch.manual_seed(0)
    P = HW * HW
    h = torch.randn(Nt, 2 * C, HW, HW, device=dev)
    conv = torch.nn.Conv2d(2 * C, C, 1).to(dev)
    W = conv.weight.detach().view(C, 2 * C)
    b = conv.bias.detach()
    G = torch.randn(Nt, C, HW, HW, device=dev)
    hr = h.clone().requires_grad_(True)

    def conv_fb():
        conv.zero_grad(set_to_none=True)
        hr.grad = None
        conv(hr).backward(G)

    t_conv_fwd = timeit(lambda: conv(h))
    t_conv_fb = timeit(conv_fb)
    t_dx_bmm = timeit(lambda: torch.bmm(W.t().expand(Nt, 2 * C, C), G.view(Nt, C, P)))
    t_dx_conv = timeit(lambda: torch.nn.grad.conv2d_input(h.shape, conv.weight, G))
    t_dw_conv = timeit(lambda: torch.nn.grad.conv2d_weight(h, conv.weight.shape, G))

    def dw_perm():
        gt = G.view(Nt, C, P).transpose(0, 1).reshape(C, Nt * P)
        ht = h.view(Nt, 2 * C, P).transpose(0, 1).reshape(2 * C, Nt * P)
        return gt @ ht.t()

    t_dw_perm = timeit(dw_perm)
    t_dw_bmm_sum = timeit(lambda: torch.bmm(G.view(Nt, C, P), h.view(Nt, 2 * C, P).transpose(1, 2)).sum(0)) \
        if Nt * C * 2 * C * 4 < 2 ** 31 else float("nan")
    t_db = timeit(lambda: G.sum((0, 2, 3)))
    dw_ref = torch.nn.grad.conv2d_weight(h, conv.weight.shape, G).view(C, 2 * C)
    err = float((dw_perm() - dw_ref).abs().max() / dw_ref.abs().max())
    print(f"{name}: conv fwd {t_conv_fwd:7.0f}  conv fwd+bwd {t_conv_fb:7.0f}  | dx bmm {t_dx_bmm:7.0f} "
          f"dx conv {t_dx_conv:7.0f} | dW conv {t_dw_conv:7.0f} dW perm+mm {t_dw_perm:7.0f} dW bmm+sum "
          f"{t_dw_bmm_sum:7.0f} | db {t_db:5.0f} us  dW relerr {err:.1e}", flush=True)
