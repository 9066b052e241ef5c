"""In-process A/B of the stem pooling kernels (knob ``pool3s2``: 0 = generic, 1 = specialised 3x3/s2/p1)
at the ResNet-50 B=256 stem shape: BN-prologue forward with argmax, fused backward (mask + BN partials).
Interleaved rounds, min microseconds, achieved TB/s of the tensors each kernel must move.

Usage (GPU): python tools/pool_ab.py [--batch 256] [--rounds 5]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402


def timeit(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    assert _lib.load(), _lib.load_error()
    ops = torch.ops.pcmp
    dev = torch.device("cuda", 0)
    N, H, W, C = a.batch, 112, 112, 64
    c = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.3
    mean, invstd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    y, idx = ops.maxpool_fwd(c, 3, 2, 1, True, sc, sh)
    dy = torch.randn(y.shape, device=dev).to(torch.bfloat16)
    nb = lambda *t: sum(x.numel() * x.element_size() for x in t)  # noqa: E731
    fwd_bytes = nb(c, y, idx)
    bwd_bytes = nb(dy, idx, c, c)    # dy + idx in, c in, g out
    best = {}
    for _ in range(a.rounds):
        for v in (0, 1):
            ops.set_knob("pool3s2", v)
            tf = timeit(lambda: ops.maxpool_fwd(c, 3, 2, 1, True, sc, sh))
            tb = timeit(lambda: ops.maxpool_bwd_bnr(dy, idx, c, mean, invstd, sc, sh, 3, 2, 1))
            b = best.setdefault(v, [1e9, 1e9])
            b[0], b[1] = min(b[0], tf), min(b[1], tb)
    ops.set_knob("pool3s2", 1)
    for v, name in ((0, "generic"), (1, "pool3s2")):
        tf, tb = best[v]
        print(f"{name:8s} maxpool_fwd(BN prologue, idx) {tf:7.1f} us {fwd_bytes / tf / 1e6:5.2f} TB/s   "
              f"maxpool_bwd_bnr {tb:7.1f} us {bwd_bytes / tb / 1e6:5.2f} TB/s")


if __name__ == "__main__":
    main()
