"""Kernel lab (not product code): the 1x1 compress conv's weight gradient, dW = sum_n dy_n h_n^T, as
MIOpen's convolution weight gradient (torch.nn.grad.conv2d_weight: NCHW -> NHWC transposes + wrw
kernel) against a batched GEMM into an (N, C, 2C) temporary + a sum over nodes, at the BASELINE
config shapes.  Times are medians of alternated rounds.

Usage: python tools/exp_compress_wgrad.py
"""
import torch

dev = torch.device("cuda:0")
SHAPES = {"north_star": (256, 512, 32), "cfg1": (128, 512, 32), "cfg2": (256, 1280, 8), "cfg3": (64, 2048, 8),
          "cfg4": (128, 1024, 16)}


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n


def main():
    for name, (Nt, C, H) in SHAPES.items():
        P = H * H
        torch.manual_seed(0)
        h = torch.randn(Nt, 2 * C, H, H, device=dev)
        dy = torch.randn(Nt, C, H, H, device=dev)
        wshape = (C, 2 * C, 1, 1)

        def miopen():
            return torch.nn.grad.conv2d_weight(h, wshape, dy)

        def bmm_sum():
            return torch.bmm(dy.view(Nt, C, P), h.view(Nt, 2 * C, P).transpose(1, 2)).sum(0).view(wshape)

        def perm_mm():  # channel-major copies of dy and h, then one GEMM with K = Nt P
            a = dy.view(Nt, C, P).permute(1, 0, 2).reshape(C, Nt * P)
            bt = h.view(Nt, 2 * C, P).permute(1, 0, 2).reshape(2 * C, Nt * P)
            return torch.mm(a, bt.t()).view(wshape)

        ref = miopen().double()
        err = float((bmm_sum().double() - ref).abs().max() / ref.abs().max())
        err2 = float((perm_mm().double() - ref).abs().max() / ref.abs().max())
        ta, tb, tc = [], [], []
        for _ in range(3):
            ta.append(timeit(miopen))
            tb.append(timeit(bmm_sum))
            tc.append(timeit(perm_mm))
        ta, tb, tc = sorted(ta)[1], sorted(tb)[1], sorted(tc)[1]
        print(f"{name:10s} Nt={Nt} C={C} P={P}: MIOpen wgrad {ta:.3f} ms, bmm + sum {tb:.3f} ms "
              f"(temp {Nt * C * 2 * C * 4 / 2**20:.0f} MiB, rel diff {err:.1e}), permute copies + mm {tc:.3f} ms "
              f"(rel diff {err2:.1e})", flush=True)
        del h, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
