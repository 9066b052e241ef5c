"""Runs the layer-1 3x3 FWD (+BN statistics) conv on the halo kernel or the implicit GEMM
(argv[1] = halo knob value) a few times, for rocprofv3 --pmc counter passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
ops = torch.ops.pcmp
ops.set_knob("halo", int(sys.argv[1]) if len(sys.argv) > 1 else 1)
mode = sys.argv[2] if len(sys.argv) > 2 else "fwd"
dev = torch.device("cuda")
x = torch.randn(256, 56, 56, 64, device=dev).to(torch.bfloat16)
w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).to(torch.bfloat16)
mean, istd = torch.zeros(64, device=dev), torch.ones(64, device=dev)
sc, sh = torch.ones(64, device=dev), torch.zeros(64, device=dev)
for _ in range(3):
    if mode == "fwd":
        ops.conv_fwd(x, w, 1, 1, None, None, False, True)
    else:
        ops.conv_dgrad_bnr(x, w, 56, 56, 1, 1, None, None, x, mean, istd, None, None, None, sc, sh)
torch.cuda.synchronize()
