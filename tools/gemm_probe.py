"""Plain-GEMM throughput of the HIP MFMA kernels vs hipBLASLt (torch.mm) on large shapes, to tell
main-loop efficiency apart from conv-specific losses (epilogues, tile quantisation, im2col).

C[M,N] = A[M,K] @ B[N,K]^T in bf16 (fp32 accumulate), uniform random operands in [-1, 1)
(cdna_hip_programming.md §5.4 rule 25: zero-filled data reads high).  Interleaved rounds, min us.

Usage: python tools/gemm_probe.py [--rounds 3] [--knobs k=v,...] [--variants 'a:k=v;b:k=v']
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

SHAPES = [(4096, 4096, 4096), (8192, 8192, 8192), (50176, 256, 2304), (200704, 128, 1152),
          (12544, 512, 4608), (4096, 3072, 768), (4096, 768, 3072)]


def timeit(fn, iters):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", default="base:")
    ap.add_argument("--no-blas", action="store_true")
    a = ap.parse_args()
    assert _lib.load(), _lib.load_error()
    ops = torch.ops.pcmp
    dev = torch.device("cuda")
    defaults = {k.split("=")[0]: int(k.split("=")[1]) for k in ops.list_knobs()}
    variants = []
    for spec in a.variants.split(";"):
        nm, _, kv = spec.partition(":")
        variants.append((nm, {k: int(v) for k, v in (i.split("=") for i in filter(None, kv.split(",")))}))
    g = torch.Generator(device=dev).manual_seed(0)
    cases = []
    for M, N, K in SHAPES:
        A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        cases.append(((M, N, K), A, B))
    res = {}
    names = [v[0] for v in variants] + ([] if a.no_blas else ["hipblaslt"])
    for _ in range(a.rounds):
        for vn, d in variants:
            for k, v in defaults.items():
                ops.set_knob(k, v)
            for k, v in d.items():
                ops.set_knob(k, v)
            for shp, A, B in cases:
                M, N, K = shp
                fn = lambda A=A, B=B, M=M, N=N, K=K: ops.conv_fwd(A.view(M, 1, 1, K), B.view(N, 1, 1, K), 1, 0,
                                                                    None, None, False, False)[0]
                res.setdefault((shp, vn), []).append(timeit(fn, a.iters))
        if not a.no_blas:
            for shp, A, B in cases:
                res.setdefault((shp, "hipblaslt"), []).append(timeit(lambda A=A, B=B: torch.mm(A, B.t()), a.iters))
    for k, v in defaults.items():
        ops.set_knob(k, v)
    print(f"{'M x N x K':24s} " + " ".join(f"{n:>20s}" for n in names))
    for shp, A, B in cases:
        M, N, K = shp
        fl = 2.0 * M * N * K
        row = [f"{min(res[(shp, n)]):8.1f}us {fl / min(res[(shp, n)]) / 1e6:5.0f}TF" for n in names]
        print(f"{M:>7d} x {N:>5d} x {K:>5d}  " + " ".join(f"{c:>20s}" for c in row))
    # correctness of the first variant on the smallest shape vs fp32
    shp, A, B = cases[0]
    M, N, K = shp
    ref = A.float() @ B.float().t()
    out = ops.conv_fwd(A.view(M, 1, 1, K), B.view(N, 1, 1, K), 1, 0, None, None, False, False)[0].view(M, N).float()
    print("max rel err vs fp32:", ((out - ref).abs().max() / ref.abs().max()).item())


if __name__ == "__main__":
    main()
