"""fp32 conv kernels of csrc/f32.hip on the ResNet-50 layer shapes (the reference's precision, TL batch
64 at 224^2 by default): time per call and TF/s of FWD (+BN stats), DGRAD and WGRAD with the 128x128
32x32x2-MFMA kernel (f32_big = 1) against the 64x64 16x16x4 kernel (f32_big = 0).

Usage: python tools/f32_conv_micro.py [batch] [knob=value,...]   (second column: those knobs instead of f32_big=0)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
ops = torch.ops.pcmp
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
# optional "knob=value,knob=value": the second column times the 32x32x2 kernel with these knobs
VARIANT = dict((k, int(v)) for k, v in (kv.split("=") for kv in sys.argv[2].split(","))) if len(sys.argv) > 2 else {}
dev = torch.device("cuda")
# name, H (input), C, K, R, stride, pad
LAYERS = [
    ("l1_1x1_64to64", 56, 64, 64, 1, 1, 0),
    ("l1_3x3_64", 56, 64, 64, 3, 1, 1),
    ("l1_1x1_64to256", 56, 64, 256, 1, 1, 0),
    ("l1_1x1_256to64", 56, 256, 64, 1, 1, 0),
    ("l2_3x3_128_s2", 56, 128, 128, 3, 2, 1),
    ("l2_3x3_128", 28, 128, 128, 3, 1, 1),
    ("l2_1x1_512to128", 28, 512, 128, 1, 1, 0),
    ("l3_3x3_256", 14, 256, 256, 3, 1, 1),
    ("l3_1x1_1024to256", 14, 1024, 256, 1, 1, 0),
    ("l3_1x1_256to1024", 14, 256, 1024, 1, 1, 0),
    ("l4_3x3_512", 7, 512, 512, 3, 1, 1),
    ("l4_1x1_2048to512", 7, 2048, 512, 1, 1, 0),
]


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


print(f"fp32 conv micro, batch {B}: us/call and TF/s, f32_big=1 (128x128 32x32x2) | f32_big=0 (64x64 16x16x4)")
tot = {0: 0.0, 1: 0.0}
for name, H, C, K, R, s, p in LAYERS:
    x = torch.randn(B, H, H, C, device=dev)
    w = torch.randn(K, R, R, C, device=dev) * (2.0 / (R * R * C)) ** 0.5
    P = (H + 2 * p - R) // s + 1
    dy = torch.randn(B, P, P, K, device=dev)
    dw = torch.empty(K, R, R, C, device=dev)
    flops = 2.0 * B * P * P * K * R * R * C
    row = f"{name:20s}"
    for mode, fn in (("fwd", lambda: ops.conv_fwd(x, w, s, p, None, None, False, True)),
                     ("dgrad", lambda: ops.conv_dgrad(dy, w, H, H, s, p, None)),
                     ("wgrad", lambda: ops.conv_wgrad(dy, x, dw, R, R, s, p, False))):
        res = []
        for big in (1, 0):
            if VARIANT and big == 0:   # second column: the 32x32x2 kernel under the VARIANT knobs instead
                olds = {k: ops.set_knob(k, v) for k, v in VARIANT.items()}
                t = timed(fn)
                for k, v in olds.items():
                    ops.set_knob(k, v)
            else:
                old = ops.set_knob("f32_big", big)
                t = timed(fn)
                ops.set_knob("f32_big", old)
            tot[big] += t
            res.append(f"{t:8.1f}us {flops / t / 1e6:5.0f}TF")
        row += f" | {mode} " + " ".join(res)
    print(row, flush=True)
print(f"total fwd+dgrad+wgrad over the listed layers: f32_big=1 {tot[1] / 1e3:.2f} ms, f32_big=0 {tot[0] / 1e3:.2f} ms")
