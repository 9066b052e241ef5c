"""Runs one memory-bound conv kernel a few times (for rocprofv3 --pmc counter passes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

_lib.load()
ops = torch.ops.pcmp
dev = torch.device("cuda")
which = sys.argv[1] if len(sys.argv) > 1 else "fwd"
x = torch.randn(256, 56, 56, 64, device=dev).to(torch.bfloat16)
w = (torch.randn(256, 1, 1, 64, device=dev) * 0.1).to(torch.bfloat16)
out = torch.empty(256 * 56 * 56 * 256, device=dev, dtype=torch.bfloat16)
src = torch.empty_like(out)
for _ in range(3):
    if which == "fwd":
        ops.conv_fwd(x, w, 1, 0, None, None, False, False)
    elif which == "fill":
        out.fill_(1.0)
    else:
        out.copy_(src)
torch.cuda.synchronize()
