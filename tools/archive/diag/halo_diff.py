"""Diagnostic: halo DGRAD (knob halo=3, halo_ovl=0) vs the implicit-GEMM DGRAD, element diffs."""
import sys, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[2]))
import torch
import pcmp  # noqa: F401
from pcmp.ops import _lib
_lib.load()
ops = torch.ops.pcmp
torch.manual_seed(0)
gpu = torch.device("cuda")
N, H, C = 20, 56, 64
rnd = lambda *s, scale=1.0: (torch.randn(*s, device=gpu) * scale).to(torch.bfloat16)
dy = rnd(N, H, H, C)
w = rnd(C, 3, 3, C, scale=(2.0 / (9 * C)) ** 0.5)
x = rnd(N, H, H, C)
mean, invstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
sc, sh = torch.randn(C, device=gpu), torch.randn(C, device=gpu) * 0.5
run = lambda: ops.conv_dgrad_bnr(dy, w, H, H, 1, 1, None, None, x, mean, invstd, None, None, None, sc, sh)
def knobbed(kn):
    old = {k: ops.set_knob(k, v) for k, v in kn.items()}
    try:
        r = run(); torch.cuda.synchronize(); return r
    finally:
        for k, v in old.items(): ops.set_knob(k, v)
base = knobbed({"halo": 0})
for kn in ({"halo": 3}, {"halo": 3, "halo_ovl": 0}, {"halo": 0}):
    for rep in range(2):
        got = knobbed(kn)
        d = (got[0].float() - base[0].float())
        bad = (d != 0)
        idx = bad.nonzero()
        print(kn, rep, "mismatch", int(bad.sum()), "max", float(d.abs().max()),
              "first", idx[:4].tolist() if len(idx) else None,
              "part sum diff", float((got[1].float().sum(0) - base[1].float().sum(0)).abs().max()))
