"""Diagnostic: the test_conv_large_shapes_8wave body on one shape, repeated; reports mask-from-x
DGRAD+BNR mismatches vs the reference with |x*sc+sh| at the mismatching elements."""
import sys, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[2]))
import torch
import pcmp  # noqa: F401
from pcmp.ops import _lib, ref
_lib.load()
ops = torch.ops.pcmp
gpu = torch.device("cuda")
N, H, W, C, K, R, s, p = (int(v) for v in sys.argv[1].split(","))
P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
rnd = lambda *sh, scale=1.0: (torch.randn(*sh, device=gpu) * scale).to(torch.bfloat16)
first = None
for it in range(int(sys.argv[2]) if len(sys.argv) > 2 else 8):
    x = rnd(N, H, W, C)
    w = rnd(K, R, R, C, scale=(2.0 / (R * R * C)) ** 0.5)
    ops.conv_fwd(x, w, s, p, None, None, False, True)
    bias = torch.randn(K, device=gpu)
    res = rnd(N, P, Q, K)
    ops.conv_fwd(x, w, s, p, bias, res, True, False)
    dy = rnd(N, P, Q, K)
    wd = rnd(K, R, R, C, scale=(2.0 / (R * R * K)) ** 0.5)
    dres = rnd(N, H, W, C)
    ops.conv_dgrad(dy, wd, H, W, s, p, dres.clone())
    xb = rnd(N, H, W, C)
    mean, invstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    sc, sh = torch.randn(C, device=gpu), torch.randn(C, device=gpu) * 0.5
    out = ops.conv_dgrad_bnr(dy, wd, H, W, s, p, None, None, xb, mean, invstd, None, None, None, sc, sh)
    out2 = ops.conv_dgrad_bnr(dy, wd, H, W, s, p, None, None, xb, mean, invstd, None, None, None, sc, sh)
    outr = ref.conv_dgrad_bnr(dy, wd, H, W, s, p, None, None, xb, mean, invstd, None, None, None, sc, sh)
    torch.cuda.synchronize()
    e = (out[0].float() - outr[0].float()).abs()
    lim = 0.02 + 0.02 * outr[0].float().abs().max().item()
    bad = e > lim
    z = (xb.float() * sc + sh)
    zf = torch.addcmul(sh.expand_as(z), xb.float(), sc.expand_as(z))
    print(it, "bad", int(bad.sum()), "max", round(float(e.max()), 3), "repeat-equal", bool(torch.equal(out[0], out2[0])),
          "|z| at bad", z[bad][:6].tolist(), flush=True)
