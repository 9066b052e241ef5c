"""In-process A/B of the BatchNorm apply kernels (v1 grid-stride vs v2 fixed-channel-group + U-deep
loads) on ResNet-50 B=256 activation shapes: microseconds, achieved TB/s, and a bitwise check that
every variant produces the same output as v1.  Variants switch through torch.ops.pcmp.set_knob.

Usage: python tools/ew_micro.py [--rounds 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

SHAPES = [(256, 112, 112, 64), (256, 56, 56, 64), (256, 56, 56, 256), (256, 28, 28, 512), (256, 14, 14, 1024),
          (256, 7, 7, 2048)]
BIG = 1 << 30
VARIANTS = [("v1", dict(bn_apply_v=1, ew_nt=0)),
            ("u4b16k", dict(bn_apply_v=2, ew_unroll=4, ew_blocks=16384, ew_nt=0)),
            ("u1all", dict(bn_apply_v=2, ew_unroll=1, ew_blocks=BIG, ew_nt=0)),
            ("u2all", dict(bn_apply_v=2, ew_unroll=2, ew_blocks=BIG, ew_nt=0)),
            ("u4all", dict(bn_apply_v=2, ew_unroll=4, ew_blocks=BIG, ew_nt=0)),
            ("u2all_nt", dict(bn_apply_v=2, ew_unroll=2, ew_blocks=BIG, ew_nt=1)),
            ("u4all_nt", dict(bn_apply_v=2, ew_unroll=4, ew_blocks=BIG, ew_nt=1))]


def timeit(fn, iters=20):
    fn()
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
    a = ap.parse_args()
    assert _lib.load(), _lib.load_error()
    ops = torch.ops.pcmp
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    defaults = {k.split("=")[0]: int(k.split("=")[1]) for k in ops.list_knobs()}
    cases = []
    for shp in SHAPES:
        C = shp[-1]
        x = torch.randn(shp, device=dev, generator=g).to(torch.bfloat16)
        x2 = torch.randn(shp, device=dev, generator=g).to(torch.bfloat16)
        dy = torch.randn(shp, device=dev, generator=g).to(torch.bfloat16)
        sc, sh = torch.rand(C, device=dev, generator=g) + 0.5, torch.randn(C, device=dev, generator=g)
        coef = torch.randn(3, C, device=dev, generator=g)
        mb = torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev)
        nb = x.numel() * 2
        cases.append((f"apply_relu {shp}", 2 * nb, lambda x=x, sc=sc, sh=sh: ops.bn_apply(x, sc, sh, None, None, None, True, None)))
        cases.append((f"apply_res_relu_bits {shp}", 3 * nb + nb // 16,
                      lambda x=x, x2=x2, sc=sc, sh=sh, mb=mb: ops.bn_apply(x, sc, sh, x2, None, None, True, mb)))
        cases.append((f"bwd_apply_mask_g {shp}", 5 * nb,
                      lambda dy=dy, x=x, x2=x2, coef=coef: ops.bn_bwd_apply(dy, x2, x, coef, None, None, True)))
        cases.append((f"bwd_apply {shp}", 3 * nb, lambda dy=dy, x=x, coef=coef: ops.bn_bwd_apply(dy, None, x, coef, None, None, False)))
    res = {}
    for r in range(a.rounds):
        for vname, knobs in VARIANTS:
            for k, v in knobs.items():
                ops.set_knob(k, v)
            for cname, nbytes, fn in cases:
                us = timeit(fn)
                res.setdefault((cname, vname), []).append(us)
    # bitwise check of every variant against v1
    mism = []
    for vname, knobs in VARIANTS:
        for cname, _, fn in cases:
            for k, v in dict(bn_apply_v=1, ew_nt=0).items():
                ops.set_knob(k, v)
            ref = fn()
            for k, v in knobs.items():
                ops.set_knob(k, v)
            out = fn()
            ref = ref if isinstance(ref, (list, tuple)) else [ref]
            out = out if isinstance(out, (list, tuple)) else [out]
            if not all(torch.equal(p, q) for p, q in zip(ref, out)):
                mism.append((cname, vname))
    for k, v in defaults.items():
        ops.set_knob(k, v)
    print(f"{'case':48s} " + " ".join(f"{v:>14s}" for v, _ in VARIANTS))
    for cname, nbytes, _ in cases:
        row = []
        for vname, _ in VARIANTS:
            us = min(res[(cname, vname)])
            row.append(f"{us:7.1f}/{nbytes / us / 1e6:4.2f}")
        print(f"{cname:48s} " + " ".join(f"{c:>14s}" for c in row))
    tot = {v: sum(min(res[(c, v)]) for c, _, _ in cases) for v, _ in VARIANTS}
    print("total us (min over rounds):", json.dumps({k: round(v, 1) for k, v in tot.items()}))
    print("bitwise mismatches vs v1:", mism)


if __name__ == "__main__":
    main()
