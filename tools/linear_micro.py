"""Time the BERT-base Linear GEMMs (M = 32 x 128 tokens) on the HIP kernels: fwd (+bias), dgrad, wgrad."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

_lib.load()
ops = torch.ops.pcmp
dev = torch.device("cuda")
M = 4096


def bench(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


for name, cin, cout in [("qkv", 768, 2304), ("attn_out", 768, 768), ("ffn1", 768, 3072), ("ffn2", 3072, 768)]:
    x = torch.randn(M, 1, 1, cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(cout, 1, 1, cin, device=dev) * 0.03).to(torch.bfloat16)
    b = torch.randn(cout, device=dev)
    dy = torch.randn(M, 1, 1, cout, device=dev).to(torch.bfloat16)
    out = torch.empty(cout, 1, 1, cin, device=dev)
    fl = 2.0 * M * cin * cout
    r = {"gemm": name, "M": M, "K": cin, "N": cout}
    for mode, fn in [("fwd", lambda: ops.conv_fwd(x, w, 1, 0, b, None, False, False)),
                     ("dgrad", lambda: ops.conv_dgrad(dy, w, 1, 1, 1, 0, None)),
                     ("wgrad", lambda: ops.conv_wgrad(dy, x, out, 1, 1, 1, 0, False))]:
        us = bench(fn)
        r[mode + "_us"] = round(us, 1)
        r[mode + "_tf"] = round(fl / us / 1e6, 1)
    print(json.dumps(r), flush=True)

# hipBLASLt (torch) on the same GEMMs: fwd = x W^T + b (addmm), dgrad = dy W, wgrad = dy^T x (fp32 out)
if "--torch" in sys.argv:
    for name, cin, cout in [("qkv", 768, 2304), ("attn_out", 768, 768), ("ffn1", 768, 3072), ("ffn2", 3072, 768)]:
        x = torch.randn(M, cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(cout, cin, device=dev) * 0.03).to(torch.bfloat16)
        b = torch.randn(cout, device=dev).to(torch.bfloat16)
        dy = torch.randn(M, cout, device=dev).to(torch.bfloat16)
        fl = 2.0 * M * cin * cout
        r = {"gemm": name, "impl": "hipblaslt"}
        for mode, fn in [("fwd", lambda: torch.addmm(b, x, w.t())),
                         ("dgrad", lambda: torch.mm(dy, w)),
                         ("wgrad", lambda: torch.mm(dy.t(), x))]:
            us = bench(fn)
            r[mode + "_us"] = round(us, 1)
            r[mode + "_tf"] = round(fl / us / 1e6, 1)
        print(json.dumps(r), flush=True)
