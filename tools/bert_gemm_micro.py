"""BERT-base GEMMs as the fused sublayers issue them (M = 32 x 128 tokens), HIP kernels vs
hipBLASLt (torch.addmm / torch.mm), min microseconds over interleaved rounds:
  fwd (bias epilogue), ffn1 fwd with the GELU epilogue (u and gelu(u) out), dgrad with the residual
  gradient added in the epilogue (qkv / ffn1), ffn2 dgrad with the GELU-backward epilogue, and
  wgrad into an fp32 gradient (split-K + reduction as the planner / autotune choose).
Usage: python tools/bert_gemm_micro.py [--rounds 3] [--knobs k=v,...]
"""
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
if "--knobs" in sys.argv:
    for kv in sys.argv[sys.argv.index("--knobs") + 1].split(","):
        k, v = kv.split("=")
        ops.set_knob(k, int(v))


def t(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


g = torch.Generator(device=dev).manual_seed(0)
cases = []
for name, cin, cout in [("qkv", 768, 2304), ("attn_out", 768, 768), ("ffn1", 768, 3072), ("ffn2", 3072, 768)]:
    x = (torch.rand(M, cin, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(cout, cin, device=dev, generator=g) * 2 - 1) * 0.03).to(torch.bfloat16)
    wt = w.t().contiguous()
    b = torch.randn(cout, device=dev, generator=g)
    dy = (torch.rand(M, cout, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    res = (torch.rand(M, cin, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    gw = torch.empty(cout, cin, device=dev)
    fl = 2.0 * M * cin * cout
    bb = b.to(torch.bfloat16)
    x4, w4, dy4, wt4 = x.view(M, 1, 1, cin), w.view(cout, 1, 1, cin), dy.view(M, 1, 1, cout), wt.view(cin, 1, 1, cout)
    if name == "ffn1":
        cases.append((f"{name}_fwd_gelu", fl, lambda x=x, w=w, b=b: ops.linear_gelu_fwd(x, w, b),
                      lambda x=x, w=w, bb=bb: torch.nn.functional.gelu(torch.addmm(bb, x, w.t()))))
        cases.append((f"{name}_fwd_plain", fl, lambda x4=x4, w4=w4, b=b: ops.conv_fwd(x4, w4, 1, 0, b, None, False, False),
                      lambda x=x, w=w, bb=bb: torch.addmm(bb, x, w.t())))
    else:
        cases.append((f"{name}_fwd", fl, lambda x4=x4, w4=w4, b=b: ops.conv_fwd(x4, w4, 1, 0, b, None, False, False),
                      lambda x=x, w=w, bb=bb: torch.addmm(bb, x, w.t())))
    if name == "ffn2":
        u = (torch.rand(M, cin, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        cases.append((f"{name}_dgrad_gelu", fl, lambda dy=dy, w=w, u=u, wt4=wt4: ops.linear_dgrad_gelu(dy, w, u, wt4.view(wt4.shape[0], -1)),
                      lambda dy=dy, w=w: torch.mm(dy, w)))
        cases.append((f"{name}_dgrad_plain", fl, lambda dy4=dy4, w4=w4, wt4=wt4: ops.conv_dgrad(dy4, w4, 1, 1, 1, 0, None, wt4),
                      lambda dy=dy, w=w: torch.mm(dy, w)))
    elif name in ("qkv", "ffn1"):
        cases.append((f"{name}_dgrad_res", fl,
                      lambda dy4=dy4, w4=w4, r=res.view(M, 1, 1, cin), wt4=wt4: ops.conv_dgrad(dy4, w4, 1, 1, 1, 0, r, wt4),
                      lambda dy=dy, w=w, r=res: torch.addmm(r, dy, w)))
    else:
        cases.append((f"{name}_dgrad", fl, lambda dy4=dy4, w4=w4, wt4=wt4: ops.conv_dgrad(dy4, w4, 1, 1, 1, 0, None, wt4),
                      lambda dy=dy, w=w: torch.mm(dy, w)))
    cases.append((f"{name}_wgrad", fl,
                  lambda dy4=dy4, x4=x4, gw4=gw.view(cout, 1, 1, cin): ops.conv_wgrad(dy4, x4, gw4, 1, 1, 1, 0, False),
                  lambda dy=dy, x=x: torch.mm(dy.t(), x)))
res_t = {}
for _ in range(ROUNDS):
    for v in ("hip", "hipblaslt"):
        for nm, fl, ours, blas in cases:
            res_t.setdefault((nm, v), []).append(t(blas if v == "hipblaslt" else ours))
tot = {"hip": 0.0, "hipblaslt": 0.0}
print(f"{'case':22s} {'hip us':>9s} {'TF':>6s} {'blaslt us':>10s} {'TF':>6s}")
for nm, fl, _, _ in cases:
    a, b_ = min(res_t[(nm, "hip")]), min(res_t[(nm, "hipblaslt")])
    tot["hip"] += a
    tot["hipblaslt"] += b_
    print(f"{nm:22s} {a:9.1f} {fl / a / 1e6:6.0f} {b_:10.1f} {fl / b_ / 1e6:6.0f}")
print(f"per layer total us: hip {tot['hip']:.1f}  hipblaslt {tot['hipblaslt']:.1f}")
