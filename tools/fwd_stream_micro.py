"""Per-shape A/B of the streaming 1x1 FWD + BatchNorm-statistics kernel (knob fwd_stream) against the
one-tile kernels on the ResNet-50 B=256 expanding 1x1 convs (conv3 of layers 1-3, the layer-1
downsample), with and without the BatchNorm-forward fold of the input.  Min microseconds over
interleaved rounds, TB/s of the ideal traffic (input + output).

Usage: python tools/fwd_stream_micro.py [--rounds 3] [--wgs 256,512]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

CASES = [   # name, N, H, K (in), C (out), act fold  (calls per step)
    ("l1_conv3_fold", 256, 56, 64, 256, True),     # 3
    ("l1_down", 256, 56, 64, 256, False),          # 1 (side stream)
    ("l2_conv3_fold", 256, 28, 128, 512, True),    # 4
    ("l3_conv3", 256, 14, 256, 1024, False),       # 6
]


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
    ap.add_argument("--wgs", default="256,512")
    a = ap.parse_args()
    assert _lib.load(), _lib.load_error()
    ops = torch.ops.pcmp
    dev = torch.device("cuda")
    variants = [("old", {"fwd_stream": 0})] + [(f"stream{w}", {"fwd_stream": 1, "bnr_stream_wgs": int(w)})
                                               for w in a.wgs.split(",")]
    print(f"{'case':18s} " + " ".join(f"{n:>22s}" for n, _ in variants))
    tot = {n: 0.0 for n, _ in variants}
    for name, N, H, K, C, fold in CASES:
        g = torch.Generator(device=dev).manual_seed(0)
        z = torch.randn(N, H, H, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(C, 1, 1, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        sc = sh = None
        if fold:
            sc, sh = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.5
        nbytes = z.numel() * 2 + N * H * H * C * 2
        best = {n: 1e30 for n, _ in variants}
        for _ in range(a.rounds):
            for n, kv in variants:
                old = {k: ops.set_knob(k, v) for k, v in kv.items()}
                best[n] = min(best[n], timeit(lambda: ops.conv_fwd(z, w, 1, 0, None, None, False, True, sc, sh)))
                for k, v in old.items():
                    ops.set_knob(k, v)
        line = f"{name:18s} "
        for n, _ in variants:
            line += f"   {best[n]:8.1f}us {nbytes / best[n] / 1e6:5.2f}TB/s"
            tot[n] += best[n]
        print(line, flush=True)
    print("total us:", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
