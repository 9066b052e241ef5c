"""BERT-base Linear GEMMs (M = 32 x 128 tokens) on the HIP kernels vs hipBLASLt, in one process:
fwd (x W^T + b) and dgrad (dY W, with the pre-transposed weight shadow the model passes), with the
plain-GEMM planner off (gemm_plan=0: round-1 dispatch) and on (autotuned kernel / K-split), plus
torch.addmm / torch.mm (hipBLASLt).  Interleaved rounds, min microseconds.

Usage: python tools/linear_micro.py [--rounds 3]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

_lib.load()
ops = torch.ops.pcmp
dev = torch.device("cuda")
M = 4096
ROUNDS = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 3


def t(fn, iters=30):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for kv in filter(None, os.environ.get("KNOBS", "").split(",")):   # e.g. KNOBS=dma_prio=1
    k, v = kv.split("=")
    ops.set_knob(k, int(v))
cases = []
g = torch.Generator(device=dev).manual_seed(0)
for name, cin, cout in [("qkv", 768, 2304), ("attn_out", 768, 768), ("ffn1", 768, 3072), ("ffn2", 3072, 768)]:
    x = torch.randn(M, 1, 1, cin, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(cout, 1, 1, cin, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    wt = w.reshape(cout, cin).t().contiguous().reshape(cin, 1, 1, cout)
    b = torch.randn(cout, device=dev, generator=g)
    dy = torch.randn(M, 1, 1, cout, device=dev, generator=g).to(torch.bfloat16)
    fl = 2.0 * M * cin * cout
    x2, w2, dy2, bb = x.view(M, cin), w.view(cout, cin), dy.view(M, cout), b.to(torch.bfloat16)
    cases.append((f"{name}_fwd", fl, lambda x=x, w=w, b=b: ops.conv_fwd(x, w, 1, 0, b, None, False, False)[0],
                  lambda x2=x2, w2=w2, bb=bb: torch.addmm(bb, x2, w2.t())))
    cases.append((f"{name}_dgrad", fl, lambda dy=dy, w=w, wt=wt: ops.conv_dgrad(dy, w, 1, 1, 1, 0, None, wt),
                  lambda dy2=dy2, w2=w2: torch.mm(dy2, w2)))
res = {}
for _ in range(ROUNDS):
    for v in ("plan0", "plan1", "hipblaslt"):
        if v != "hipblaslt":
            ops.set_knob("gemm_plan", 0 if v == "plan0" else 1)
        for nm, fl, ours, blas in cases:
            res.setdefault((nm, v), []).append(t(blas if v == "hipblaslt" else ours))
ops.set_knob("gemm_plan", 1)
# numerics: planned result vs hipBLASLt (bf16 out)
for nm, fl, ours, blas in cases:
    a, r = ours().float().reshape(-1), blas().float().reshape(-1)
    err = ((a - r).norm() / r.norm()).item()
    row = {v: round(min(res[(nm, v)]), 1) for v in ("plan0", "plan1", "hipblaslt")}
    row.update({"gemm": nm, "tf_plan1": round(fl / min(res[(nm, 'plan1')]) / 1e6), "rel_err_vs_blas": f"{err:.1e}"})
    print(json.dumps(row), flush=True)
print("plans:", sorted(ops.gemm_plans()))
