"""Run one plain GEMM (or one conv case) a few times on the HIP kernels, for rocprofv3 --pmc passes.

Usage: python tools/gemm_one.py --shape 8192,8192,8192 [--knobs dma32=0] [--plan 2] [--iters 5]
       python tools/gemm_one.py --conv l3_3x3_256:fwd
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="8192,8192,8192")
ap.add_argument("--knobs", default="")
ap.add_argument("--plan", type=int, default=-1, help="plan_force kind (2 = 8-wave 256x256 DMA)")
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--conv", default=None, help="name:mode of a tools/gemm_knob_ab.py case")
a = ap.parse_args()
assert _lib.load(), _lib.load_error()
ops = torch.ops.pcmp
for kv in filter(None, a.knobs.split(",")):
    k, v = kv.split("=")
    ops.set_knob(k, int(v))
dev = torch.device("cuda")
if a.conv:
    sys.argv = [sys.argv[0]]
    import gemm_knob_ab as gk  # noqa: E402
    name, mode = a.conv.split(":")
    cases = [c for c in gk.build_cases(mode, name) if c[0].split()[0] == mode or c[0].startswith(mode + " ")]
    fn = cases[0][3]
else:
    M, N, K = map(int, a.shape.split(","))
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    if a.plan >= 0:
        ops.set_knob("plan_force", a.plan)
    fn = lambda: ops.conv_fwd(A.view(M, 1, 1, K), B.view(N, 1, 1, K), 1, 0, None, None, False, False)
fn()
torch.cuda.synchronize()
for _ in range(a.iters):
    fn()
torch.cuda.synchronize()
print("ok")
