"""Parameter plumbing shared by every autograd Function of the framework.

* **Compute weights.**  Parameters are fp32 masters.  Kernels consume a compute-dtype copy
  (bf16 on the GPU).  When the model's parameters are flattened (:class:`pcmp.utils.flat.FlatParams`),
  ``p._shadow`` is a view into one contiguous bf16 buffer that the fused optimizer kernel
  rewrites in the same pass as the fp32 update; otherwise the copy is cached per ``p._version``.

* **Gradient sinks.**  With flattened parameters each parameter carries ``p.main_grad``, an fp32
  view into the flat gradient buffer (whose slices are the DDP all-reduce buckets).  Backward
  kernels write weight gradients straight into that view (overwrite on the first write of a
  step, accumulate afterwards) and then fire ``p._grad_ready_hook`` so the data-parallel
  engine can launch the bucket's all-reduce while the rest of backward runs.  Without a sink
  the gradient is returned to autograd as usual.
"""
from __future__ import annotations

import os
from typing import Callable

import torch

# Global weight generation: bumped whenever parameters or BN running statistics change through a
# path that does not touch the tensors' version counters (fused optimizer kernels, BN-statistics
# updates inside training forwards).  Derived caches (inference BN folding) key on it.
WEIGHT_GEN = [0]


def bump_weight_gen():
    WEIGHT_GEN[0] += 1


def compute_weight(p: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    sh = getattr(p, "_shadow", None)
    if sh is not None and sh.dtype == dtype:
        return sh
    if p.dtype == dtype:
        return p.detach()
    cache = getattr(p, "_shadow_cache", None)
    if cache is None or cache[0] != p._version or cache[1].dtype != dtype or cache[1].device != p.device:
        cache = (p._version, p.detach().to(dtype).contiguous())
        p._shadow_cache = cache
    return cache[1]


def compute_weight_t(p: torch.Tensor, dtype: torch.dtype):
    """Transposed [C,R,S,K] compute weight for DGRAD from the flat arena, or None (the kernel
    then transposes per call)."""
    owner = getattr(p, "_flat_owner", None)
    if owner is None or dtype != torch.bfloat16:
        return None
    from . import _lib
    if _lib.backend() == "torch":
        return None    # the reference backend computes DGRAD from w; the arena's class-blocked form is HIP-only
    return owner.transposed(p)


def emit_grad(p: torch.Tensor | None, compute: Callable[[torch.Tensor, bool], None]):
    """Produce the gradient of ``p``.  ``compute(out, accumulate)`` fills an fp32 tensor.

    Returns the tensor to hand back to autograd, or None when it went into a sink.
    """
    if p is None or not p.requires_grad:
        return None
    mg = getattr(p, "main_grad", None)
    if mg is not None:
        fresh = getattr(p, "_grad_fresh", True)
        compute(mg, not fresh)
        p._grad_fresh = False
        hook = getattr(p, "_grad_ready_hook", None)
        if hook is not None:
            hook(p)
        return None
    out = torch.empty(p.shape, dtype=torch.float32, device=p.device)
    compute(out, False)
    return out if p.dtype == torch.float32 else out.to(p.dtype)


def needs_grad(p) -> bool:
    return p is not None and isinstance(p, torch.Tensor) and p.requires_grad


def sink_or_temp(p: torch.Tensor | None):
    """For kernels that write a small gradient (BN gamma/beta) directly: returns
    (out_tensor_or_None, accumulate, finish) where ``finish()`` returns the autograd value."""
    if p is None or not p.requires_grad:
        return None, False, (lambda: None)
    mg = getattr(p, "main_grad", None)
    if mg is not None:
        acc = not getattr(p, "_grad_fresh", True)

        def finish():
            p._grad_fresh = False
            hook = getattr(p, "_grad_ready_hook", None)
            if hook is not None:
                hook(p)
            return None
        return mg, acc, finish
    tmp = torch.empty(p.shape, dtype=torch.float32, device=p.device)
    return tmp, False, (lambda: tmp)


# ------------------------------------------------------------------------------------------------
# Weight-gradient side stream.  Within a block's backward, WGRAD(L) and DGRAD(L) both depend only on
# the layer's output gradient, so WGRAD runs on a second HIP stream and fills the CUs that the
# DGRAD chain leaves idle (small grids, tile tails, the latency-bound BN finalize launches).  The
# compute stream joins the side stream at the end of every backward pass (autograd engine
# callback), and the data-parallel bucket launch orders the all-reduce after both streams.
# PCMP_WGRAD_STREAM=0 keeps everything on one stream.
_SIDE: dict = {}
_JOIN_QUEUED = [False]
_ENV: dict = {}


def refresh_env() -> None:
    """Re-read the side-stream switches (PCMP_WGRAD_STREAM, PCMP_SIDE_WGRAD_WGS,
    PCMP_SIDE_WGRAD_WGS_LINEAR); they are cached because run_on_side is on the per-kernel host path
    (A/B tools call this after editing os.environ)."""
    _ENV["side"] = os.environ.get("PCMP_WGRAD_STREAM", "1") != "0"
    for key, var, dflt in (("wgs", "PCMP_SIDE_WGRAD_WGS", 384), ("wgs_linear", "PCMP_SIDE_WGRAD_WGS_LINEAR", 160)):
        try:
            _ENV[key] = max(0, int(os.environ.get(var, str(dflt))))
        except ValueError:
            _ENV[key] = dflt


refresh_env()


def side_stream_enabled() -> bool:
    return _ENV["side"]


def active_streams(device):
    """(compute stream, wgrad stream) pair in use on ``device`` this backward, or ()."""
    return _SIDE.get(("active", torch.device(device).index), ())


def _join(main, side, key):
    main.wait_stream(side)
    _SIDE.pop(key, None)
    _JOIN_QUEUED[0] = False


def fork_side(fn: Callable[[], object], keep_alive):
    """Run ``fn`` on the device's side stream, ordered after the compute stream's work so far, and
    return ``(result, event)``: the compute stream must ``wait_event(event)`` (``join_side``) before
    it consumes the result.  For independent branches inside one autograd node (a residual block's
    downsample conv next to its main branch)."""
    dev = keep_alive[0].device
    main = torch.cuda.current_stream(dev)
    side = _SIDE.get(dev.index)
    if side is None:
        side = _SIDE[dev.index] = torch.cuda.Stream(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        out = fn()
    for t in keep_alive:
        if t is not None:
            t.record_stream(side)
    ev = torch.cuda.Event()
    ev.record(side)
    return out, ev


def join_side(result, ev):
    """Make the compute stream wait for a ``fork_side`` result and register its tensors with it."""
    ts = [t for t in (result if isinstance(result, (tuple, list)) else (result,)) if isinstance(t, torch.Tensor)]
    main = torch.cuda.current_stream(ts[0].device)
    main.wait_event(ev)
    for t in ts:
        t.record_stream(main)
    return result


def _side_wgrad_wgs() -> int:
    """Split-K workgroup target of side-stream WGRADs (``PCMP_SIDE_WGRAD_WGS``, default 384; 0 keeps
    the per-shape autotune, which times each WGRAD alone)."""
    return _ENV["wgs"]


# per device: [side stream, ring of fork events, ring position].  run_on_side runs ~50 times per
# training step, so its host cost counts (BERT-base's eager step is launch-bound on a slow host,
# profiles/r4_bert_host_prof.txt): raw current-stream get / set instead of Stream objects and the
# stream context manager, and recycled events instead of one new Event per fork.  A recycled
# event is re-recorded only after 256 later forks -- the wait enqueued on it long since resolved.
_SIDE_CTX: dict = {}
_NEV = 256


def _side_ctx(idx: int):
    c = _SIDE_CTX.get(idx)
    if c is None:
        side = _SIDE.get(idx)
        if side is None:
            side = _SIDE[idx] = torch.cuda.Stream(idx)
        c = _SIDE_CTX[idx] = [side, [torch.cuda.Event() for _ in range(_NEV)], 0]
    return c


def run_on_side(fn: Callable[[], None], keep_alive, linear: bool = False) -> None:
    """Run ``fn`` (kernel launches) on the device's WGRAD stream, ordered after the compute stream's
    work so far; ``keep_alive`` tensors are recorded on the side stream for the caching allocator.
    ``linear``: Linear-layer WGRADs (BERT's M = 4096-token reductions) take the split-K workgroup
    target PCMP_SIDE_WGRAD_WGS_LINEAR (160: fewer splits and reduce launches -- +1.8 % BERT-base
    step vs 384, profiles/r5_bert_wgs_ab.txt) instead of the conv target."""
    idx = keep_alive[0].get_device()
    c = _side_ctx(idx)
    side = c[0]
    cur = torch._C._cuda_getCurrentStream(idx)   # (stream id, device index, device type)
    ev = c[1][c[2]]
    c[2] = (c[2] + 1) % _NEV
    ev.record()                                   # on the compute stream (current)
    side.wait_event(ev)
    if not _JOIN_QUEUED[0]:
        main = torch.cuda.Stream(stream_id=cur[0], device_index=cur[1], device_type=cur[2])
        key = ("active", idx)
        _SIDE[key] = (main, side)
        _JOIN_QUEUED[0] = True
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _join(main, side, key))
    wgs = _ENV["wgs_linear" if linear else "wgs"]
    torch._C._cuda_setStream(stream_id=side.stream_id, device_index=idx, device_type=side.device_type)
    try:
        if wgs:
            prev = torch.ops.pcmp.set_knob("wgrad_wgs", wgs)
            try:
                fn()
            finally:
                torch.ops.pcmp.set_knob("wgrad_wgs", prev)   # keep a PCMP_KNOBS=wgrad_wgs=N setting
        else:
            fn()
    finally:
        torch._C._cuda_setStream(stream_id=cur[0], device_index=cur[1], device_type=cur[2])
    for t in keep_alive:
        t.record_stream(side)
