"""Per-shape A/B of the streaming DGRAD + BN-backward-reduce kernel (knob bnr_stream) against the
one-tile kernels, on the ResNet-50 B=256 layer-1/2 configurations the backward sends to
conv_dgrad_bnr (dz fold, dual BN, full / sub-sampled residual, mask bits / recomputed).
Interleaved rounds, min microseconds, achieved TB/s of the ideal traffic.

Usage: python tools/bnr_stream_micro.py [--rounds 3] [--wgs 512,1024,2048]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402,F401

# name, N, H, K (dz channels), C (dx channels), fold, dual, resid, mask  (calls per ResNet-50 step)
CASES = [
    ("l1b1_conv1_fold_dual", 256, 56, 64, 256, True, True, "full", "bits"),     # 1
    ("l1b2_conv1_fold", 256, 56, 64, 256, True, False, "full", "bits"),         # 1
    ("l2b0_conv1_fold_sub", 256, 56, 128, 256, True, False, "sub", "bits"),     # 1
    ("l1_conv3_fold_mfx", 256, 56, 256, 64, True, False, "none", "mfx"),        # 3
    ("l2_conv1", 256, 28, 128, 512, False, False, "full", "bits"),              # 2
    ("l2b1_conv1_dual", 256, 28, 128, 512, False, True, "full", "bits"),        # 1
    ("l3b0_conv1_sub", 256, 28, 256, 512, False, False, "sub", "bits"),         # 1
    ("l2_conv3_mfx", 256, 28, 512, 128, False, False, "none", "mfx"),           # (K=512: not eligible)
    ("l3_conv1", 256, 14, 256, 1024, False, False, "full", "bits"),             # 4
    ("l3b1_conv1_dual", 256, 14, 256, 1024, False, True, "full", "bits"),       # 1
    ("l3_conv3_mfx", 256, 14, 1024, 256, False, False, "none", "mfx"),          # (K=1024: not eligible)
]


def operands(dev, N, H, K, C, fold, dual, resid, mask):
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(torch.bfloat16)

    dy = rnd(N, H, H, K)
    fx = coef = None
    if fold:
        fx = rnd(N, H, H, K)
        coef = torch.stack([torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.05,
                            torch.randn(K, device=dev) * 0.1]).contiguous()
    w = rnd(K, 1, 1, C, scale=0.05)
    x = rnd(N, H, H, C)
    mean, istd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    x2 = mean2 = istd2 = None
    if dual:
        x2, mean2, istd2 = rnd(N, H, H, C), torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    res = rnd(N, H, H, C) if resid == "full" else (rnd(N, H // 2, H // 2, C) if resid == "sub" else None)
    bits = msc = msh = None
    if mask == "bits":
        bits = torch.randint(0, 256, (N * H * H * C // 8,), device=dev, dtype=torch.uint8)
    else:
        msc, msh = torch.randn(C, device=dev), torch.randn(C, device=dev) * 0.5
    nbytes = dy.numel() * 2 * (2 if fold else 1) + x.numel() * 2 * (2 + (1 if dual else 0)) + \
        (res.numel() * 2 if res is not None else 0) + (bits.numel() if bits is not None else 0)
    return (dy, w, H, H, 1, 0, res, None, x, mean, istd, x2, mean2, istd2, msc, msh, None, bits, fx, coef,
            resid == "sub"), nbytes


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--wgs", default="512")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    assert _lib.load(), _lib.load_error()
    ops = torch.ops.pcmp
    dev = torch.device("cuda")
    variants = [("old", {"bnr_stream": 0})] + [(f"stream{w}", {"bnr_stream": 1, "bnr_stream_wgs": int(w)})
                                               for w in a.wgs.split(",")]
    print(f"{'case':26s} " + " ".join(f"{n:>22s}" for n, _ in variants))
    tot = {n: 0.0 for n, _ in variants}
    for case in CASES:
        if a.only and not any(o in case[0] for o in a.only.split(",")):
            continue
        args, nbytes = operands(dev, *case[1:])
        best = {n: 1e30 for n, _ in variants}
        for _ in range(a.rounds):
            for n, kv in variants:
                old = {k: ops.set_knob(k, v) for k, v in kv.items()}
                best[n] = min(best[n], timeit(lambda: ops.conv_dgrad_bnr(*args)))
                for k, v in old.items():
                    ops.set_knob(k, v)
        line = f"{case[0]:26s} "
        for n, _ in variants:
            line += f"   {best[n]:8.1f}us {nbytes / best[n] / 1e6:5.2f}TB/s"
            tot[n] += best[n]
        print(line, flush=True)
        del args
        torch.cuda.empty_cache()
    print("total us:", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
