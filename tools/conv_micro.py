"""Time individual implicit-GEMM conv shapes (HIP kernels vs MIOpen via torch) for kernel tuning.

Usage: python tools/conv_micro.py [--modes fwd,dgrad,wgrad] [--torch] [--iters 20]
Shapes are ResNet-50 @ B=256 representatives (see tools/conv_roofline.py for the full table).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

SHAPES = [  # name, N, H, W, C, K, R, stride, pad
    ("l1_1x1_64to256", 256, 56, 56, 64, 256, 1, 1, 0),
    ("l1_1x1_256to64", 256, 56, 56, 256, 64, 1, 1, 0),
    ("l1_3x3_64", 256, 56, 56, 64, 64, 3, 1, 1),
    ("l2_3x3_128", 256, 28, 28, 128, 128, 3, 1, 1),
    ("l2_1x1_128to512", 256, 28, 28, 128, 512, 1, 1, 0),
    ("l3_3x3_256", 256, 14, 14, 256, 256, 3, 1, 1),
    ("l3_1x1_1024to256", 256, 14, 14, 1024, 256, 1, 1, 0),
    ("l4_3x3_512", 256, 7, 7, 512, 512, 3, 1, 1),
    ("l3_1x1_256to1024", 256, 14, 14, 256, 1024, 1, 1, 0),
    ("l4_1x1_2048to512", 256, 7, 7, 2048, 512, 1, 1, 0),
    ("l4_1x1_512to2048", 256, 7, 7, 512, 2048, 1, 1, 0),
    ("stem_7x7", 256, 224, 224, 8, 64, 7, 2, 3),
    # GEMM-like probes for the 8-wave BM=256 kernel (BN=256 variant)
    ("x_3x3_256_28", 256, 28, 28, 256, 256, 3, 1, 1),
    ("x_1x1_512to512_28", 256, 28, 28, 512, 512, 1, 1, 0),
]


def bench(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="fwd,dgrad,wgrad")
    ap.add_argument("--torch", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    _lib.load()
    ops = torch.ops.pcmp
    dev = torch.device("cuda")
    for name, N, H, W, C, K, R, s, p in SHAPES:
        if a.only and a.only not in name:
            continue
        P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(K, R, R, C, device=dev) * 0.05).to(torch.bfloat16)
        dy = torch.randn(N, P, Q, K, device=dev).to(torch.bfloat16)
        out = torch.empty(K, R, R, C, device=dev)
        flops = 2.0 * N * P * Q * K * R * R * C
        for mode in a.modes.split(","):
            if mode == "dgrad" and name.startswith("stem"):
                continue
            if mode == "dgrad_bnr":
                if name.startswith("stem"):
                    continue
                xm = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
                mu, isd = torch.zeros(C, device=dev), torch.ones(C, device=dev)
                fn = lambda: ops.conv_dgrad_bnr(dy, w, H, W, s, p, None, None, xm, mu, isd, None, None, None, isd, mu)
            elif mode == "fwd":
                fn = lambda: ops.conv_fwd(x, w, s, p, None, None, False, True)
            elif mode == "dgrad":
                fn = lambda: ops.conv_dgrad(dy, w, H, W, s, p, None)
            else:
                fn = lambda: ops.conv_wgrad(dy, x, out, R, R, s, p, False)
            t = bench(fn, a.iters)
            rec = {"shape": name, "mode": mode, "us": round(t * 1e6, 1), "tflops": round(flops / t / 1e12, 1)}
            if a.torch:
                xc = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
                wc = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
                dyc = dy.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
                if mode == "fwd":
                    tf = lambda: torch.nn.functional.conv2d(xc, wc, None, s, p)
                elif mode.startswith("dgrad"):
                    tf = lambda: torch.nn.grad.conv2d_input(xc.shape, wc, dyc, s, p)
                else:
                    tf = lambda: torch.nn.grad.conv2d_weight(xc, wc.shape, dyc, s, p)
                tt = bench(tf, a.iters)
                rec["torch_us"] = round(tt * 1e6, 1)
                rec["speedup"] = round(tt / t, 2)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
