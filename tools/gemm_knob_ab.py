"""In-process A/B of implicit-GEMM kernel variants (switched with torch.ops.pcmp.set_knob) on the
ResNet-50 B=256 convolution shapes with their training epilogues: FWD + BN statistics, DGRAD + fused
BN-backward reduction (mask bits, residual gradient), WGRAD into an fp32 gradient.  Interleaved
rounds, min microseconds, achieved TB/s / TF/s, and the max abs difference against the first
variant's output.

Usage: python tools/gemm_knob_ab.py --variants 'base:;new:dma32=0' [--only l1_] [--rounds 3]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

# name, N, H, W, Cin, Cout, R, stride, pad
SHAPES = [
    ("stem_s2d_4x4_16to64", 256, 115, 115, 16, 64, 4, 1, 0),
    ("l1_1x1_64to256", 256, 56, 56, 64, 256, 1, 1, 0),
    ("l1_1x1_256to64", 256, 56, 56, 256, 64, 1, 1, 0),
    ("l1_3x3_64", 256, 56, 56, 64, 64, 3, 1, 1),
    ("l2_1x1_512to128", 256, 28, 28, 512, 128, 1, 1, 0),
    ("l2_1x1_128to512", 256, 28, 28, 128, 512, 1, 1, 0),
    ("l2_3x3_128", 256, 28, 28, 128, 128, 3, 1, 1),
    ("l3_1x1_1024to256", 256, 14, 14, 1024, 256, 1, 1, 0),
    ("l3_1x1_256to1024", 256, 14, 14, 256, 1024, 1, 1, 0),
    ("l3_3x3_256", 256, 14, 14, 256, 256, 3, 1, 1),
    ("l4_3x3_512", 256, 7, 7, 512, 512, 3, 1, 1),
    ("l4_1x1_2048to512", 256, 7, 7, 2048, 512, 1, 1, 0),
    ("l4_1x1_512to2048", 256, 7, 7, 512, 2048, 1, 1, 0),
]


def timeit(fn, iters):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def build_cases(modes, only):
    ops = torch.ops.pcmp
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    cases = []
    for name, N, H, W, C, K, R, s, p in SHAPES:
        if only and not any(o in name for o in only.split(",")):
            continue
        P = (H + 2 * p - R) // s + 1
        x = (torch.randn(N, H, W, C, device=dev, generator=g)).to(torch.bfloat16)
        w = (torch.randn(K, R, R, C, device=dev, generator=g) * (2.0 / (R * R * C)) ** 0.5).to(torch.bfloat16)
        dy = torch.randn(N, P, P, K, device=dev, generator=g).to(torch.bfloat16)
        flops = 2.0 * N * P * P * K * R * R * C
        if "fwd" in modes:
            byts = (x.numel() + w.numel() + dy.numel()) * 2
            cases.append((f"fwd_stats {name}", flops, byts,
                          lambda x=x, w=w, s=s, p=p: ops.conv_fwd(x, w, s, p, None, None, False, True)))
        if "dgrad" in modes:
            xb = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
            res = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
            mean = torch.randn(C, device=dev, generator=g) * 0.1
            istd = torch.rand(C, device=dev, generator=g) + 0.5
            bits = torch.randint(0, 256, (N * H * W * C // 8,), device=dev, dtype=torch.uint8, generator=g)
            byts = (dy.numel() + 3 * xb.numel()) * 2 + bits.numel()

            def dg(dy=dy, w=w, H=H, W=W, s=s, p=p, xb=xb, res=res, mean=mean, istd=istd, bits=bits):
                return ops.conv_dgrad_bnr(dy, w, H, W, s, p, res.clone() if s == 2 else res, None, xb, mean, istd,
                                          None, None, None, None, None, None, bits)
            cases.append((f"dgrad_bnr {name}", flops, byts, dg))
            if s == 1 and R == 1 and K < C:
                # dual BN-reduce form (the DGRAD into a block whose tail has a downsample BN): the main
                # and downsample BN inputs, both reductions, residual gradient, mask bits
                x2 = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
                mean2 = torch.randn(C, device=dev, generator=g) * 0.1
                istd2 = torch.rand(C, device=dev, generator=g) + 0.5

                def dg2(dy=dy, w=w, H=H, W=W, p=p, xb=xb, res=res, mean=mean, istd=istd, bits=bits, x2=x2,
                        mean2=mean2, istd2=istd2):
                    return ops.conv_dgrad_bnr(dy, w, H, W, 1, p, res, None, xb, mean, istd, x2, mean2, istd2,
                                              None, None, None, bits)
                cases.append((f"dgrad_bnr2 {name}", flops, byts + x2.numel() * 2, dg2))
            if s == 1 and R == 3:
                # intermediate-layer form (the model's conv2 DGRAD): mask recomputed from x, no residual
                msc, msh = torch.rand(C, device=dev, generator=g) + 0.5, torch.randn(C, device=dev, generator=g) * 0.1

                def dgm(dy=dy, w=w, H=H, W=W, p=p, xb=xb, mean=mean, istd=istd, msc=msc, msh=msh):
                    return ops.conv_dgrad_bnr(dy, w, H, W, 1, p, None, None, xb, mean, istd, None, None, None, msc, msh)
                cases.append((f"dgrad_bnr_mfx {name}", flops, (dy.numel() + 2 * xb.numel()) * 2, dgm))
        if "wgrad" in modes:
            out = torch.zeros(K, R, R, C, device=dev)
            byts = (x.numel() + dy.numel()) * 2 + out.numel() * 4
            cases.append((f"wgrad {name}", flops, byts,
                          lambda dy=dy, x=x, out=out, R=R, s=s, p=p: (ops.conv_wgrad(dy, x, out, R, R, s, p, False), out)[1]))
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True, help="'name:k=v,k=v;name2:...'")
    ap.add_argument("--modes", default="fwd,dgrad,wgrad")
    ap.add_argument("--only", default=None)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    assert _lib.load(), _lib.load_error()
    ops = torch.ops.pcmp
    defaults = {k.split("=")[0]: int(k.split("=")[1]) for k in ops.list_knobs()}
    variants = []
    for spec in a.variants.split(";"):
        nm, _, kv = spec.partition(":")
        d = {}
        for item in filter(None, kv.split(",")):
            k, v = item.split("=")
            d[k] = int(v)
        variants.append((nm, d))

    def setv(d):
        for k, v in defaults.items():
            ops.set_knob(k, v)
        for k, v in d.items():
            ops.set_knob(k, v)

    cases = build_cases(a.modes, a.only)
    res = {}
    for _ in range(a.rounds):
        for vn, d in variants:
            setv(d)
            for cn, _, _, fn in cases:
                res.setdefault((cn, vn), []).append(timeit(fn, a.iters))
    diffs = {}
    for cn, _, _, fn in cases:
        outs = []
        for vn, d in variants:
            setv(d)
            o = fn()
            o = o[0] if isinstance(o, (list, tuple)) else o
            outs.append(o.float().clone())
        for (vn, _), o in zip(variants, outs):
            diffs[(cn, vn)] = (o - outs[0]).abs().max().item()
    setv({})
    print(f"{'case':34s} " + " ".join(f"{vn:>24s}" for vn, _ in variants))
    tot = {vn: 0.0 for vn, _ in variants}
    for cn, fl, by, _ in cases:
        row = []
        for vn, _ in variants:
            us = min(res[(cn, vn)])
            tot[vn] += us
            row.append(f"{us:7.1f}us {by / us / 1e6:4.2f}TB {fl / us / 1e6:5.0f}TF d{diffs[(cn, vn)]:.0e}")
        print(f"{cn:34s} " + " ".join(f"{c:>24s}" for c in row))
    print("total us:", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
