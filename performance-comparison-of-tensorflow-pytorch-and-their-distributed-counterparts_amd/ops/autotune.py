"""Per-shape backend choice for plain Linear GEMMs: the MFMA implicit-GEMM kernels vs hipBLASLt.

The task's rule for MI355X: hand-written MFMA kernels for the fused hot ops, hipBLASLt only for
plain library GEMMs.  A BERT-sized Linear (M = 4096 tokens, K/N in 768..3072) forward (x W^T + b)
or input gradient (dY W) is exactly such a plain GEMM; hipBLASLt runs several of those shapes
1.3-1.6x faster than the implicit-GEMM kernel (profiles/r1_bert_gemm_vs_hipblaslt.txt).  So the
first call of each (op, M, K, N) times both on the live stream (cudnn.benchmark-style) and caches
the faster.  Everything with a fused epilogue (conv + BN statistics / BN-backward reduction) and
every weight gradient (fp32 into the flat gradient buffer) stays on the hand-written kernels.

Only for M >= ``MIN_ROWS`` (small-batch heads keep the deterministic in-house kernels), never while
a graph is being captured, and ``PCMP_LINEAR_BLAS=0`` disables the hipBLASLt candidate.
"""
from __future__ import annotations

import os

import torch

MIN_ROWS = 1024
_CACHE: dict = {}


def _enabled() -> bool:
    return os.environ.get("PCMP_LINEAR_BLAS", "1") != "0"


def _time(fn, reps=3) -> float:
    fn()   # warm (library heuristics, allocations)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e)


def pick(key, ours, blas) -> str:
    """Return "ours" or "blas" for this GEMM key (timing both on first use)."""
    if not _enabled() or key[1] < MIN_ROWS:
        return "ours"
    hit = _CACHE.get(key)
    if hit is not None:
        return hit
    if torch.cuda.is_current_stream_capturing():
        return "ours"
    choice = "blas" if _time(blas) < _time(ours) else "ours"
    _CACHE[key] = choice
    return choice


def choices() -> dict:
    return dict(_CACHE)
