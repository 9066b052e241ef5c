"""Per-op GPU time of one ResNet training step, with a roofline estimate for every call.

Every ``K.<op>`` dispatch (pcmp/ops/kernels.py) is bracketed by CUDA events on the current stream;
after a few warm-up steps one step is recorded, then calls are aggregated by (op, shapes).  For each
group it prints total us, count, achieved TB/s (tensor bytes in + out) and TFLOP/s (conv ops), and
the roofline floor max(bytes / BW, flops / PEAK) so the gap per op class is visible.

Usage (GPU): python tools/layer_profile.py [--model resnet50] [--batch 256] [--top 60]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import kernels  # noqa: E402

BW = 5.3e12      # achievable HBM3E streaming bandwidth (B/s) measured for copies on MI355X
PEAK = 2.3e15    # dense bf16 MFMA peak (FLOP/s) at the sustained clock


def _nbytes(v):
    if isinstance(v, torch.Tensor):
        return v.numel() * v.element_size()
    if isinstance(v, (list, tuple)):
        return sum(_nbytes(t) for t in v)
    return 0


def _shape(v):
    return tuple(v.shape) if isinstance(v, torch.Tensor) else (v if isinstance(v, (int, float, bool)) or v is None else "?")


def conv_flops(name, args):
    if name == "conv_fwd":
        x, w, s, p = args[0], args[1], args[2], args[3]
        N, H, W, C = x.shape
        Kc, R, S, _ = w.shape
        P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - S) // s + 1
        return 2.0 * N * P * Q * Kc * R * S * C
    if name in ("conv_dgrad", "conv_dgrad_bnr"):
        dy, w = args[0], args[1]
        N, P, Q, Kc = dy.shape
        _, R, S, C = w.shape
        return 2.0 * N * P * Q * Kc * R * S * C
    if name == "conv_wgrad":
        dy, x, R, S = args[0], args[1], args[3], args[4]
        N, P, Q, Kc = dy.shape
        return 2.0 * N * P * Q * Kc * R * S * x.shape[3]
    return 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()

    from pcmp.models import resnet
    from pcmp.ops import cross_entropy
    from pcmp.optim import SGD
    from pcmp.utils.flat import FlatParams

    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = getattr(resnet, a.model)(num_classes=1000).to(dev).train()
    flat = FlatParams(model.parameters())
    opt = SGD(flat, lr=0.1, momentum=0.9, weight_decay=5e-5)
    x = torch.rand(a.batch, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (a.batch,), device=dev)

    rec = [None]
    K = kernels.K
    for name in kernels.OP_NAMES:
        inner = getattr(K, name)

        def wrapped(*args, _inner=inner, _name=name):
            if rec[0] is None:
                return _inner(*args)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = _inner(*args)
            e1.record()
            # keep only sizes: holding the tensors would defeat the caching allocator's reuse and the
            # fresh (driver-cleared) allocations would then be timed as part of the ops
            nb = sum(_nbytes(v) for v in args) + _nbytes(out)
            shapes = tuple(_shape(v) for v in args if isinstance(v, torch.Tensor))[:3]
            rec[0].append((_name, shapes, nb, conv_flops(_name, args), e0, e1))
            return out

        setattr(K, name, wrapped)

    def step():
        opt.zero_grad()
        loss = cross_entropy(model.forward_logits(x), y)
        loss.backward()
        opt.step()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    rec[0] = []
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    step()
    t1.record()
    torch.cuda.synchronize()
    calls = rec[0]
    rec[0] = None
    step_ms = t0.elapsed_time(t1)

    groups = collections.OrderedDict()
    by_op = collections.defaultdict(lambda: [0.0, 0.0, 0])
    tot_us = tot_floor = 0.0
    for name, shapes, nb, fl, e0, e1 in calls:
        us = e0.elapsed_time(e1) * 1e3
        floor = max(nb / BW, fl / PEAK) * 1e6
        key = (name, shapes)
        g = groups.setdefault(key, [0.0, 0, nb, fl, floor])
        g[0] += us
        g[1] += 1
        by_op[name][0] += us
        by_op[name][1] += floor
        by_op[name][2] += 1
        tot_us += us
        tot_floor += floor
    print(f"step {step_ms:.2f} ms (event-bracketed), {len(calls)} dispatched ops, op time {tot_us / 1e3:.2f} ms, "
          f"roofline floor {tot_floor / 1e3:.2f} ms")
    print("\nby op:  total_ms  floor_ms  calls")
    for name, (us, fl, n) in sorted(by_op.items(), key=lambda kv: -kv[1][0]):
        print(f"  {name:18s} {us / 1e3:8.2f} {fl / 1e3:8.2f} {n:6d}")
    print("\nby (op, shapes): total_us  x  us/call  floor_us  gap_us  TB/s  TF/s")
    rows = sorted(groups.items(), key=lambda kv: -(kv[1][0] - kv[1][4] * kv[1][1]))
    for (name, shapes), (us, n, nb, fl, floor) in rows[: a.top]:
        per = us / n
        print(f"  {us:8.0f} x{n:2d} {per:8.1f} {floor:8.1f} {us - floor * n:8.0f}  {nb / per / 1e6:5.2f} "
              f"{fl / per / 1e6:7.1f}  {name} {shapes}")


if __name__ == "__main__":
    main()
