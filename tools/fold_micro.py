"""Per-shape cost of the BatchNorm-backward fold (ResNet-50, B=256): for every 1x1 conv whose dy is a
BN-backward output, time (a) bn_bwd_apply + the unfused DGRAD (its normal kernel choice) + WGRAD on dz
against (b) the folded DGRAD / WGRAD that form dz while staging.  CUDA events, interleaved rounds.

Usage (GPU): python tools/fold_micro.py [--rounds 5]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
ops = torch.ops.pcmp


def timeit(fn, reps=5):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    # (name, spatial, K = dy channels, C = dgrad output channels, into_prev)
    shapes = []
    for li, (hw, c) in enumerate([(56, 64), (28, 128), (14, 256), (7, 512)], 1):
        shapes.append((f"l{li} conv3 dz3", hw, 4 * c, c, False))
        shapes.append((f"l{li} conv1 dz1", hw, c, 4 * c, True))
    print(f"{'shape':16s} {'apply':>8s} {'dgrad':>8s} {'dgradF':>8s} {'wgrad':>8s} {'wgradF':>8s}   "
          f"{'crit unf':>9s} {'crit fold':>9s} {'side unf':>9s} {'side fold':>9s}  (us)")
    for name, hw, K, C, into_prev in shapes:
        N = a.batch
        bf = torch.bfloat16
        g = torch.randn(N, hw, hw, K, device=dev).to(bf)
        x = (torch.randn(N, hw, hw, K, device=dev) + 0.5).to(bf)
        coef = torch.stack([torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.05,
                            torch.randn(K, device=dev) * 0.1]).contiguous()
        w = (torch.randn(K, 1, 1, C, device=dev) * 0.05).to(bf)
        wt = w.permute(3, 1, 2, 0).contiguous()
        xb = torch.randn(N, hw, hw, C, device=dev).to(bf)
        mean, istd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
        xin = torch.randn(N, hw, hw, C, device=dev).to(bf)
        out = torch.empty(K, 1, 1, C, device=dev)
        if into_prev:   # residual + mask bits (the DGRAD into the previous block's tail)
            res = torch.randn(N, hw, hw, C, device=dev).to(bf)
            bits = torch.randint(0, 256, (N * hw * hw * C // 8,), device=dev, dtype=torch.uint8)
            extra = (res, None, xb, mean, istd, None, None, None, None, None, wt, bits)
        else:           # mask recomputed from x (the DGRAD into an intermediate BN)
            sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
            extra = (None, None, xb, mean, istd, None, None, None, sc, sh, wt, None)
        dz = ops.bn_bwd_apply(g, None, x, coef, None, None, False)[0]
        res_ = {k: [] for k in ("apply", "dgrad", "dgradF", "wgrad", "wgradF")}
        for _ in range(a.rounds):
            res_["apply"].append(timeit(lambda: ops.bn_bwd_apply(g, None, x, coef, None, None, False)))
            res_["dgrad"].append(timeit(lambda: ops.conv_dgrad_bnr(dz, w, hw, hw, 1, 0, *extra)))
            res_["dgradF"].append(timeit(lambda: ops.conv_dgrad_bnr(g, w, hw, hw, 1, 0, *extra, x, coef)))
            res_["wgrad"].append(timeit(lambda: ops.conv_wgrad(dz, xin, out, 1, 1, 1, 0, False)))
            res_["wgradF"].append(timeit(lambda: ops.conv_wgrad(g, xin, out, 1, 1, 1, 0, False, x, coef)))
        m = {k: sorted(v)[len(v) // 2] for k, v in res_.items()}
        print(f"{name:16s} {m['apply']:8.1f} {m['dgrad']:8.1f} {m['dgradF']:8.1f} {m['wgrad']:8.1f} {m['wgradF']:8.1f}   "
              f"{m['apply'] + m['dgrad']:9.1f} {m['dgradF']:9.1f} {m['wgrad']:9.1f} {m['wgradF']:9.1f}", flush=True)


if __name__ == "__main__":
    main()
